#!/bin/bash
# A/B of library builds on the GPU box: for each round, copy every variant .so over libvqa.so in turn and run the
# default bench (no CPU baseline / roofline legs). Usage: tools/ab_libs.sh ROUNDS lib1.so lib2.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
LIB=vae-based-music--deep-generative-models_amd/libvqa.so
cp $LIB gpurun_out/libvqa_base.so
ROUNDS=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq $ROUNDS); do
  for v in gpurun_out/libvqa_base.so "$@"; do
    cp "$v" $LIB
    out=$(timeout -k 10 240 python bench.py --no-cpu-baseline --no-roofline --no-prior --no-fp32 --steps 40 --warmup 5 2>gpurun_out/ab/err.log) || { echo "bench failed for $v"; cp gpurun_out/libvqa_base.so $LIB; exit 1; }
    echo "$(basename $v) $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"])')"
  done
done
cp gpurun_out/libvqa_base.so $LIB
