#!/bin/bash
# round-4 GPU call X: the whole -m gpu suite + smoke on the merged library (DP test ranks taking turns on the
# shared GPU); the residual-block occupancy-3 variant's tests; the step A/B (product vs the library before this
# round's second kernel set vs the occupancy-3 variant)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4x}
TAG=$T LIMIT=${LIMIT:-900} tools/r4_call.sh \
  "dp:python -u -m pytest tests/test_gpu_dp.py -v -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider" \
  "all:python -u -m pytest tests -v -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider" \
  "smoke:python -c \"import __graft_entry__ as g; g.smoke()\"" \
  "occ3_tests:tools/lib_tests.sh variants/r4occ3.so tests/test_gpu_resblock.py" \
  "step_ab:tools/ab_libs.sh 2 variants/r4base.so variants/r4occ3.so"
