#!/bin/bash
# round-4 GPU call Q: DP rank vs one process per level: reconstruction, spectral-loss gradient, target waveform
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4q}
TAG=$T LIMIT=${LIMIT:-500} tools/r4_call.sh \
  "full_graph:VQA_DP_BATCH=32 VQA_DP_PHASES=step1 VQA_DIAG_CONFIG=cfg2 python -u tools/dp_diag.py host 4 graph"
