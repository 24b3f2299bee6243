#!/bin/bash
# Round-4 split argmin rows per wave (VQA_ARGMIN_RT 4 / 6 / 8): kernel times, then the VQ tests on each variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4amrt
tools/lib_ab.sh "python tools/argmin_time.py" variants/am_rt6.so variants/am_rt8.so > gpurun_out/r4amrt/time.log 2>&1 || exit 1
tools/lib_ab.sh "python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_vq.py 2>&1 | tail -2" variants/am_rt6.so variants/am_rt8.so > gpurun_out/r4amrt/tests.log 2>&1
