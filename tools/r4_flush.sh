#!/bin/bash
# Round-4: partial-row flush granularity (VQA_FLUSH_MB) A/B on the default step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4flush
tools/ab_env.sh 2 "VQA_FLUSH_MB=0" "VQA_FLUSH_MB=24" "VQA_FLUSH_MB=48" "VQA_FLUSH_MB=96" "VQA_FLUSH_MB=192" > gpurun_out/r4flush/ab.log 2>&1
