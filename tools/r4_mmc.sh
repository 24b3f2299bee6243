#!/bin/bash
# Round-4: max-memory-clause scheduling for the residual-block file only vs for every source: GPU tests of the
# whole-library variant, then a 5-round step A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r4mmc
mkdir -p $OUT
tools/lib_ab.sh "python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_resblock.py tests/test_gpu_conv.py tests/test_gpu_vq.py tests/test_gpu_spectral.py 2>&1 | tail -1" variants/all_mmc.so > $OUT/tests.log 2>&1 || exit 1
tools/ab_libs.sh 5 variants/rb_max-memory-clause.so variants/all_mmc.so > $OUT/step_ab.log 2>&1
