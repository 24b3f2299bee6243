#!/bin/bash
# round-4 GPU call L: local-gradient reproducibility probes (same process / side stream / fresh process / after
# another batch shape), cfg2_short and cfg2 at B = 32, bf16
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4l}
TAG=$T LIMIT=${LIMIT:-400} tools/r4_call.sh \
  "short_bf16:python -u tools/det_probe.py cfg2_short bf16 2" \
  "short_fp32:python -u tools/det_probe.py cfg2_short fp32 2" \
  "full_bf16:python -u tools/det_probe.py cfg2 bf16 32"
