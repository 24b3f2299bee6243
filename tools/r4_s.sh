#!/bin/bash
# round-4 GPU call S: a single process's step gradient, repeated, alone and beside a busy second process
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4s}
TAG=$T LIMIT=${LIMIT:-300} tools/r4_call.sh \
  "alone:python -u tools/dp_hog.py cfg2 bf16 32 4 --alone" \
  "hog:python -u tools/dp_hog.py cfg2 bf16 32 6" \
  "hog_serial:VQA_LEVEL_STREAMS=0 python -u tools/dp_hog.py cfg2 bf16 32 6"
