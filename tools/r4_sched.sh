#!/bin/bash
# Round-4: AMDGPU scheduler strategies for the residual-block kernels (variants of vqa_resblock.hip only):
# resblock tests on each variant, then the step A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r4sched
mkdir -p $OUT
tools/lib_ab.sh "python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_resblock.py 2>&1 | tail -1" variants/rb_max-ilp.so variants/rb_max-memory-clause.so > $OUT/tests.log 2>&1 || exit 1
tools/ab_libs.sh 3 variants/rb_max-ilp.so variants/rb_max-memory-clause.so > $OUT/step_ab.log 2>&1
