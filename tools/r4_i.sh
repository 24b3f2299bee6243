#!/bin/bash
# round-4 GPU call I: bisect the DP exchange-contract failure of r4h (step layout vs the EMA/quantizer kernel set)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4i}
TEST='tests/test_gpu_dp.py::test_exchange_stream_contract_both_sides[eager]'
TAG=$T LIMIT=${LIMIT:-400} tools/r4_call.sh \
  "prod:python -u -m pytest '$TEST' -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "prod_r3layout:VQA_STEP_LAYOUT=r3 python -u -m pytest '$TEST' -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "base_lib:tools/lib_tests.sh variants/r4base.so '$TEST'" \
  "serial_levels:VQA_LEVEL_STREAMS=0 python -u -m pytest '$TEST' -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider"
