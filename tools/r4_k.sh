#!/bin/bash
# round-4 GPU call K: is a launch configuration (persistent grids sized by the occupancy API) dependent on the
# process's history? occupancy probe; the exchange-contract test alone vs after the conv tests in one process
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4k}
TEST='tests/test_gpu_dp.py::test_exchange_stream_contract_both_sides[eager]'
TAG=$T LIMIT=${LIMIT:-400} tools/r4_call.sh \
  "occ:tools/probe/occ_probe" \
  "after_conv:python -u -m pytest tests/test_gpu_conv.py '$TEST' -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "after_cond:python -u -m pytest tests/test_gpu_cond.py '$TEST' -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "after_dp_fp32:python -u -m pytest 'tests/test_gpu_dp.py::test_dp2_matches_single_process_global_batch[cfg2_short-fp32-eager]' '$TEST' -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider"
