#!/bin/bash
# round-4 GPU call AA: residual-block forward with relu(x) staged in LDS (variants/r4fwdrelu.so) vs the round-3
# staging (variants/r4fwdraw.so): the resblock tests on the new form, per-kernel times at T = 32768 (d = 1..27),
# the step A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4aa}
mkdir -p gpurun_out/$T
TAG=$T LIMIT=${LIMIT:-600} tools/r4_call.sh \
  "tests:tools/lib_tests.sh variants/r4fwdrelu.so 'tests/test_gpu_resblock.py tests/test_gpu_train.py'" \
  "kernel:tools/kt_fwd.sh variants/r4fwdraw.so raw gpurun_out/$T && tools/kt_fwd.sh variants/r4fwdrelu.so relu gpurun_out/$T && tools/kt_fwd.sh variants/r4fwdraw.so raw2 gpurun_out/$T && tools/kt_fwd.sh variants/r4fwdrelu.so relu2 gpurun_out/$T" \
  "step_ab:tools/ab_libs.sh 3 variants/r4fwdraw.so variants/r4fwdrelu.so"
