#!/bin/bash
# round-4 GPU call O: DP rank vs one process, with the level statistics (code counts, EMA sums) compared too
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4o}
TAG=$T LIMIT=${LIMIT:-400} tools/r4_call.sh \
  "full_graph:VQA_DP_BATCH=32 VQA_DP_PHASES=step1 VQA_DIAG_CONFIG=cfg2 python -u tools/dp_diag.py host 3 graph" \
  "short_eager:python -u tools/dp_diag.py host 8 eager"
