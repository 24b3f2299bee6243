#!/bin/bash
# A/B of a variant library on the GPU box: its GPU tests, the step A/B (tools/ab_libs.sh) and a serialised
# kernel trace of each library (per-kernel durations). The product library is restored at the end.
# Usage: tools/try_lib.sh VARIANT.so "TEST FILES" TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=vae-based-music--deep-generative-models_amd/libvqa.so
V=$1; TESTS=$2; TAG=${3:-v}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cp $L $OUT/base.so
cp "$V" $L
timeout -k 10 500 python -u -m pytest $TESTS -q -x -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/variant_tests.log 2>&1
rc=$?
tail -3 $OUT/variant_tests.log
cp $OUT/base.so $L
if [ $rc -ne 0 ]; then echo "tests failed ($rc)"; exit $rc; fi
for lib in base variant; do
  if [ $lib = variant ]; then cp "$V" $L; fi
  VQA_LEVEL_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$lib -o t -- \
    python bench.py --no-cpu-baseline --no-roofline --no-prior --no-fp32 --steps 10 > $OUT/bench_serial_$lib.json 2>$OUT/err_$lib || { cp $OUT/base.so $L; echo "trace failed"; exit 1; }
  python tools/step_breakdown.py $OUT/trace_$lib/t_kernel_trace.csv > $OUT/breakdown_$lib.txt
  find $OUT/trace_$lib -name "*kernel_trace.csv" -size +20M -delete
done
cp $OUT/base.so $L
head -40 $OUT/breakdown_base.txt > $OUT/b.txt; head -40 $OUT/breakdown_variant.txt > $OUT/v.txt; paste $OUT/b.txt $OUT/v.txt | cut -c1-200
tools/ab_libs.sh 2 "$V"
