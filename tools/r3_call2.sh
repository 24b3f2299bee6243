#!/bin/bash
# product tests touched this round + resblock variant tests / sweep / step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r3ab2; mkdir -p $OUT
export TMPDIR=/tmp
true
true
L=vae-based-music--deep-generative-models_amd/libvqa.so
cp $L $OUT/base.so
for v in "$@"; do
  cp "$v" $L
  timeout -k 10 400 python -u -m pytest tests/test_gpu_resblock.py -q -x -m gpu -k "backward" --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_$(basename $v .so).log 2>&1
  rc=$?; echo "$(basename $v) tests: $(tail -1 $OUT/tests_$(basename $v .so).log)"
  cp $OUT/base.so $L
  [ $rc -ne 0 ] && exit $rc
done
for v in $OUT/base.so "$@"; do
  cp "$v" $L
  timeout -k 10 150 python tools/resblock_sweep.py --T 32768 8192 --reps 20 2>/dev/null | cut -c1-62 > $OUT/sw_$(basename $v .so).txt || { cp $OUT/base.so $L; exit 1; }
done
cp $OUT/base.so $L
paste $OUT/sw_base.txt $(for v in "$@"; do echo $OUT/sw_$(basename $v .so).txt; done) | sed 's/fused fwd//g' | cut -c1-250
tools/ab_libs.sh ${ABR:-3} "$@"
