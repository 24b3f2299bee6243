#!/bin/bash
# round-4 GPU call P: the DP-rank vs one-process gradient difference per module (full per-rank size, graph)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4p}
TAG=$T LIMIT=${LIMIT:-500} tools/r4_call.sh \
  "full_graph:VQA_DP_BATCH=32 VQA_DP_PHASES=step1 VQA_DIAG_CONFIG=cfg2 python -u tools/dp_diag.py host 4 graph"
