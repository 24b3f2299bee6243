#!/bin/bash
# round-4 GPU call M: where do DP ranks' local gradients differ from one process? (tools/dp_diag.py: per rank,
# the bucket at exchange entry vs a single-process local gradient, and the exchanged sum)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4m}
TAG=$T LIMIT=${LIMIT:-400} tools/r4_call.sh \
  "short_graph:python -u tools/dp_diag.py host 6 graph" \
  "short_eager:python -u tools/dp_diag.py host 4 eager" \
  "full_graph:VQA_DP_BATCH=32 VQA_DP_PHASES=step1 VQA_DIAG_CONFIG=cfg2 python -u tools/dp_diag.py host 2 graph"
