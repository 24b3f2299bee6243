#!/bin/bash
# Round-4: max-memory-clause scheduling for one more source besides the residual blocks (conv / spectral /
# VQ+decoder tail+conv ends): 5-round step A/B against the shipped library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r4mmc2
mkdir -p $OUT
tools/ab_libs.sh 5 variants/mmc_conv.so variants/mmc_spec.so variants/mmc_vq.so > $OUT/step_ab.log 2>&1
