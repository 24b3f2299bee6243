#!/bin/bash
# Round-3 GPU call: the DP tests, then a variant library's resblock tests + sweep + step A/B (tools/try_variant.sh).
# Usage: tools/r3_try.sh VARIANT.so [extra test files run with the variant]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3
V=$1; shift
if [ -n "$DP" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py -v -s --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/r3/dp.log 2>&1
  echo "dp tests rc=$?"; grep -E "^(FAIL|ok) |PASSED|FAILED|passed|failed" gpurun_out/r3/dp.log | grep -v "^ok" | tail -30
fi
tools/try_variant.sh "$V" "tests/test_gpu_resblock.py $*" ${SWEEP_T:-32768 8192 2048}
