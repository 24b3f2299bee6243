#!/bin/bash
# round-4 GPU call N: which layers' local gradients differ between a DP rank and one process (dp_diag reports
# the worst parameters), eager on the short form and graph at the full per-rank size
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4n}
TAG=$T LIMIT=${LIMIT:-400} tools/r4_call.sh \
  "short_eager:python -u tools/dp_diag.py host 8 eager" \
  "full_graph:VQA_DP_BATCH=32 VQA_DP_PHASES=step1 VQA_DIAG_CONFIG=cfg2 python -u tools/dp_diag.py host 2 graph" \
  "full_graph_serial:VQA_LEVEL_STREAMS=0 VQA_DP_BATCH=32 VQA_DP_PHASES=step1 VQA_DIAG_CONFIG=cfg2 python -u tools/dp_diag.py host 2 graph"
