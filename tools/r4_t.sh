#!/bin/bash
# round-4 GPU call T: the busy-neighbour race with the caching allocator off (every tensor its own allocation,
# no block reuse across or within streams) and with the round-3 step layout
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4t}
TAG=$T LIMIT=${LIMIT:-400} tools/r4_call.sh \
  "nocache:PYTORCH_NO_CUDA_MEMORY_CACHING=1 python -u tools/dp_hog.py cfg2 bf16 32 5" \
  "r3layout:VQA_STEP_LAYOUT=r3 python -u tools/dp_hog.py cfg2 bf16 32 5"
