#!/bin/bash
# Round-end measurement on the GPU box: bench line under rocprofv3 kernel-trace stats, then two PMC passes
# (FETCH_SIZE, WRITE_SIZE; separate runs) for the dominant kernel's HBM traffic. Usage: tools/round_profile.sh TAG
set -o pipefail
TAG=${1:-r1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o f -- \
  python bench.py --no-graph --no-roofline --no-cpu-baseline --no-fp32 --no-prior --steps 2 --warmup 1 > "$OUT/pmc_fetch.log" 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o w -- \
  python bench.py --no-graph --no-roofline --no-cpu-baseline --no-fp32 --no-prior --steps 2 --warmup 1 > "$OUT/pmc_write.log" 2>&1 || { echo "write pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_mfma" -o m -- \
  python bench.py --no-graph --no-roofline --no-cpu-baseline --no-fp32 --no-prior --steps 2 --warmup 1 > "$OUT/pmc_mfma.log" 2>&1 || { echo "mfma pass failed"; exit 1; }
python tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" profiles/pmc_traffic.json "$OUT/pmc_mfma" > "$OUT/pmc.json" || exit 1
cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"
# per-kernel durations are taken with the levels serialised (VQA_LEVEL_STREAMS=0): with the levels on
# concurrent streams a kernel's duration includes the share of the GPU its neighbours take
VQA_LEVEL_STREAMS=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o t -- \
  python bench.py --no-fp32 > "$OUT/bench_serial.json" 2> "$OUT/bench_serial.err" || { echo "serial bench failed"; exit 1; }
# the bench line itself: default settings, no profiler
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; exit 1; }
find "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_mfma" -name "*counter_collection.csv" -size +20M -delete
find "$OUT/trace" -name "*kernel_trace.csv" -size +20M -delete
python tools/stats_summary.py "$OUT/trace/t_kernel_stats.csv" "$OUT/bench_serial.json" "$OUT/bench.json" > "$OUT/summary.md"
cat "$OUT/bench.json"
