#!/bin/bash
# GPU test files given as arguments (one pytest process), then the bench line. First failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r3t}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest "$@" -q -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { grep -E "FAILED|Error|passed|failed" $OUT/tests.log | tail -20; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
