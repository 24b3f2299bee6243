#!/bin/bash
# round-4 GPU call J: bisect the fp32 cfg2_short DP mismatch (isolated runs: product, r3 layout, base library)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4j}
TEST='tests/test_gpu_dp.py::test_dp2_matches_single_process_global_batch[cfg2_short-fp32-eager]'
TEST2='tests/test_gpu_dp.py::test_dp2_matches_single_process_global_batch'
TAG=$T LIMIT=${LIMIT:-400} tools/r4_call.sh \
  "prod:python -u -m pytest '$TEST' -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "prod_r3layout:VQA_STEP_LAYOUT=r3 python -u -m pytest '$TEST' -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "base_lib:tools/lib_tests.sh variants/r4base.so '$TEST'" \
  "serial_levels:VQA_LEVEL_STREAMS=0 python -u -m pytest '$TEST' -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "dp_file_base:tools/lib_tests.sh variants/r4base.so tests/test_gpu_dp.py" \
  "dp_file_r3layout:VQA_STEP_LAYOUT=r3 python -u -m pytest tests/test_gpu_dp.py -q -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider"
