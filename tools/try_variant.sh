#!/bin/bash
# Try a variant libvqa on the GPU box: GPU tests with it, the resblock sweep before / after, then the step A/B.
# The product library is restored at the end. Usage: tools/try_variant.sh VARIANT.so "TEST FILES" [SWEEP_T...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=vae-based-music--deep-generative-models_amd/libvqa.so
V=$1; TESTS=$2; shift 2
SW=${*:-32768 16384}
cp $L gpurun_out/base.so
cp "$V" $L
timeout -k 10 400 python -u -m pytest $TESTS -q -x -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/variant_tests.log 2>&1
rc=$?
tail -3 gpurun_out/variant_tests.log
if [ $rc -ne 0 ]; then cp gpurun_out/base.so $L; echo "tests failed ($rc)"; exit $rc; fi
cp gpurun_out/base.so $L
timeout -k 10 120 python tools/resblock_sweep.py --T $SW --reps 20 2>/dev/null | cut -c1-62 > gpurun_out/sw_base.txt || exit 1
cp "$V" $L
timeout -k 10 120 python tools/resblock_sweep.py --T $SW --reps 20 2>/dev/null | cut -c1-62 > gpurun_out/sw_new.txt || { cp gpurun_out/base.so $L; exit 1; }
cp gpurun_out/base.so $L
paste gpurun_out/sw_base.txt gpurun_out/sw_new.txt | cut -c1-150
tools/ab_libs.sh 2 "$V"
