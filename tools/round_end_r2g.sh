#!/bin/bash
# Round-2 closing run: LN-fusion A/B, every GPU test file, smoke, the bench line, the prior bench legs and the
# prior's kernel stats. Each GPU step has its own limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r2g
export TMPDIR=/tmp
tools/ab_prior_ln.sh | tee gpurun_out/r2g/ab_ln.txt || exit 1
STEP_TIMEOUT=420 tools/gpu_tests.sh tests/test_gpu_*.py > gpurun_out/r2g/gpu_tests.txt 2>&1 || { tail -20 gpurun_out/r2g/gpu_tests.txt; exit 1; }
grep -E "exit=|passed|failed" gpurun_out/r2g/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r2g/bench.json 2> gpurun_out/r2g/bench.err || { echo "bench failed"; exit 1; }
cat gpurun_out/r2g/bench.json
timeout -k 10 600 python tools/bench_prior.py > gpurun_out/r2g/prior_bench.json 2> gpurun_out/r2g/prior_bench.err || { echo "prior bench failed"; exit 1; }
cat gpurun_out/r2g/prior_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2g/pprof -o p -- \
  python tools/bench_prior.py --no-cpu --only train > gpurun_out/r2g/pprof.json 2> gpurun_out/r2g/pprof.err || { echo "prior profile failed"; exit 1; }
find gpurun_out/r2g/pprof -name "*kernel_trace.csv" -size +20M -delete
echo done
