#!/bin/bash
# A/B of environment settings on the GPU box: each argument is an env assignment list ("A=1 B=2" or "-").
# Usage: tools/ab_env.sh ROUNDS "VAR=x" "VAR=y" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROUNDS=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq $ROUNDS); do
  for e in "$@"; do
    envs=(); [ "$e" != "-" ] && read -ra envs <<< "$e"
    out=$(env "${envs[@]}" timeout -k 10 240 python bench.py --no-cpu-baseline --no-roofline --no-prior --no-fp32 --steps 40 --warmup 5 2>gpurun_out/ab/err.log) || { echo "bench failed for $e"; exit 1; }
    echo "$e $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"])')"
  done
done
