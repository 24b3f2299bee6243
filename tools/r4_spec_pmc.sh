#!/bin/bash
# PMC of the spectral pair kernels on the variant library variants/spec_new.so (in-tree library restored after).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=vae-based-music--deep-generative-models_amd/libvqa.so
cp $L /tmp/spec_base.so
cp variants/spec_new.so $L
tools/pmc_kernel.sh r4sp_new spec_pair -- python tools/spec_one.py 5 > gpurun_out/r4sp_new_pmc.txt 2>&1
rc=$?
cp /tmp/spec_base.so $L
exit $rc
