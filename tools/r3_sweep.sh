#!/bin/bash
# per-kernel sweep of resblock variants (no tests: timing-only builds allowed). Usage: tools/r3_sweep.sh V.so...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=vae-based-music--deep-generative-models_amd/libvqa.so
OUT=gpurun_out/r3sw; mkdir -p $OUT; cp $L $OUT/base.so
for v in $OUT/base.so "$@"; do
  cp "$v" $L
  timeout -k 10 150 python tools/resblock_sweep.py --T ${SWEEP_T:-32768 8192} --reps 20 2>/dev/null | cut -c1-62 > $OUT/sw_$(basename $v .so).txt || { cp $OUT/base.so $L; exit 1; }
done
cp $OUT/base.so $L
paste $OUT/sw_base.txt $(for v in "$@"; do echo $OUT/sw_$(basename $v .so).txt; done) | sed 's/fused fwd//g' | cut -c1-250
