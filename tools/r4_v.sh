#!/bin/bash
# round-4 GPU call V: the two-process nondeterminism vs the number of hardware queues per process (one queue per
# process: every stream of a process on one queue, no oversubscription of the hardware queues)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4v}
TAG=$T LIMIT=${LIMIT:-400} tools/r4_call.sh \
  "hog_q1:GPU_MAX_HW_QUEUES=1 python -u tools/dp_hog.py cfg2 bf16 32 5" \
  "dp_q1:GPU_MAX_HW_QUEUES=1 VQA_DP_BATCH=32 VQA_DP_PHASES=step1 VQA_DIAG_CONFIG=cfg2 python -u tools/dp_diag.py host 3 graph" \
  "hog_q2:GPU_MAX_HW_QUEUES=2 python -u tools/dp_hog.py cfg2 bf16 32 5"
