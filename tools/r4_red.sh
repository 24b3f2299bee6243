#!/bin/bash
# Round-4 partial-reduction A/B: reduce launches of one config-2 step per library variant, then the step A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4red
# the in-tree library is the w16u8 build (the new default)
tools/lib_ab.sh "python -u tools/reduce_time.py" variants/red_base.so variants/red_w4u8.so variants/red_w8u8.so \
  variants/red_w8u16.so variants/red_w16u16.so > gpurun_out/r4red/reduce_time.log 2>&1 || exit 1
tools/ab_libs.sh 2 variants/red_base.so variants/red_w8u16.so > gpurun_out/r4red/step_ab.log 2>&1
