#!/bin/bash
# Step A/B of environment settings on one library, alternating rounds: tools/env_ab.sh ROUNDS "ENV_A" "ENV_B" ...
# (an empty string = the defaults); prints ms/step per setting and round.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROUNDS=$1; shift
for r in $(seq 1 $ROUNDS); do
  for e in "$@"; do
    ms=$(env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-prior --no-fp32 --no-roofline --steps 30 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])")
    echo "round $r [${e:-default}] $ms ms/step"
  done
done
