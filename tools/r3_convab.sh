#!/bin/bash
# conv sweep of the product library and each variant (timing-only variants allowed: no tests)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=vae-based-music--deep-generative-models_amd/libvqa.so
OUT=gpurun_out/r3cv; mkdir -p $OUT; cp $L $OUT/base.so
for v in $OUT/base.so "$@"; do
  cp "$v" $L
  timeout -k 10 200 python tools/conv_sweep.py > $OUT/cs_$(basename $v .so).txt 2>&1 || { cp $OUT/base.so $L; exit 1; }
  head -2 $OUT/cs_$(basename $v .so).txt | tail -1
done
cp $OUT/base.so $L
