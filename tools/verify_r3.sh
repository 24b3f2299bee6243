#!/bin/bash
# Round-3 verification run: every GPU test file, smoke, the bench line. First failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r3v}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
STEP_TIMEOUT=420 tools/gpu_tests.sh tests/test_gpu_*.py > gpurun_out/$TAG/gpu_tests.txt 2>&1 || { tail -20 gpurun_out/$TAG/gpu_tests.txt; exit 1; }
grep -E "exit=|passed|failed" gpurun_out/$TAG/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "bench failed"; exit 1; }
cat gpurun_out/$TAG/bench.json
