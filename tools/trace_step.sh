#!/bin/bash
# Kernel trace of a short bench run (no roofline replays, no CPU leg) for tools/step_breakdown.py.
# Usage: tools/trace_step.sh TAG [extra bench.py args]
set -o pipefail
TAG=${1:-trace}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o t -- \
  python bench.py --steps 6 --warmup 2 --no-roofline --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
python tools/step_breakdown.py "$OUT/t_kernel_trace.csv" > "$OUT/step.txt"
cat "$OUT/bench.json"; head -40 "$OUT/step.txt"
