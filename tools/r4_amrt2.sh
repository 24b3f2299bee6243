#!/bin/bash
# Round-4 split argmin with RT = 8 for N >= 262,144: VQ tests and kernel times on the new library, step A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4amrt2
tools/lib_ab.sh "python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_vq.py 2>&1 | tail -3; python tools/argmin_time.py" variants/am_rt.so > gpurun_out/r4amrt2/tests_time.log 2>&1 || exit 1
tools/ab_libs.sh 5 variants/am_rt.so > gpurun_out/r4amrt2/step_ab.log 2>&1
