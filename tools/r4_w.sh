#!/bin/bash
# round-4 GPU call W: where (item, sample) and how large the reconstruction differences of a DP rank are
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4w}
TAG=$T LIMIT=${LIMIT:-400} tools/r4_call.sh \
  "dp:VQA_DP_BATCH=32 VQA_DP_PHASES=step1 VQA_DIAG_CONFIG=cfg2 python -u tools/dp_diag.py host 4 graph"
