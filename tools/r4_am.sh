#!/bin/bash
# Round-4 argmin: PMC issue/wait breakdown at N = 262144.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tools/pmc_kernel.sh r4am argmin_split -- python tools/argmin_time.py 262144 > gpurun_out/r4am_pmc.txt 2>&1
