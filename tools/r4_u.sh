#!/bin/bash
# round-4 GPU call U: guard bands around every device allocation of one train step (out-of-bounds writes)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4u}
TAG=$T LIMIT=${LIMIT:-300} tools/r4_call.sh \
  "full_bf16:VQA_LEVEL_STREAMS=0 python -u tools/guard_probe.py cfg2 bf16 32" \
  "short_fp32:VQA_LEVEL_STREAMS=0 python -u tools/guard_probe.py cfg2_short fp32 2"
