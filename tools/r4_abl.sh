#!/bin/bash
# Round-4 timing-only ablations of the default step (upper bounds of what each part could still buy).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4abl
for r in 1 2; do
  for a in none no_reduce no_spectral no_argmin; do
    out=$(timeout -k 10 240 python tools/ablate_step.py $a --no-cpu-baseline --no-roofline --no-prior --steps 40 --warmup 5 2>gpurun_out/r4abl/err_$a.log) || { echo "failed: $a"; exit 1; }
    echo "$a $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"])')"
  done
done > gpurun_out/r4abl/ab.log 2>&1
