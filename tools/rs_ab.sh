#!/bin/bash
# Residual-block variants on the GPU box: the resblock GPU tests with each variant, the per-kernel sweep of each
# library (tools/resblock_sweep.py) and the step A/B (tools/ab_libs.sh). Usage: tools/rs_ab.sh V1.so [V2.so ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=vae-based-music--deep-generative-models_amd/libvqa.so
OUT=gpurun_out/rs_ab
mkdir -p $OUT
cp $L $OUT/base.so
for v in "$@"; do
  cp "$v" $L
  timeout -k 10 300 python -u -m pytest tests/test_gpu_resblock.py -q -x -m gpu --timeout 250 --timeout-method thread -p no:cacheprovider > $OUT/tests_$(basename $v .so).log 2>&1
  rc=$?; echo "$(basename $v) tests: $(tail -1 $OUT/tests_$(basename $v .so).log)"
  cp $OUT/base.so $L
  [ $rc -ne 0 ] && exit $rc
done
for v in $OUT/base.so "$@"; do
  cp "$v" $L
  timeout -k 10 150 python tools/resblock_sweep.py --T ${SWEEP_T:-32768 8192 2048} --reps 20 2>/dev/null | cut -c1-62 > $OUT/sw_$(basename $v .so).txt || { cp $OUT/base.so $L; exit 1; }
done
cp $OUT/base.so $L
paste $OUT/sw_base.txt $(for v in "$@"; do echo $OUT/sw_$(basename $v .so).txt; done) | sed 's/fused fwd//g'
tools/ab_libs.sh 2 "$@"
