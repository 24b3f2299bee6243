#!/bin/bash
# round-4 GPU call Y: cross-lane shuffle results alone / on 4 streams / beside a busy second process
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4y}
mkdir -p gpurun_out/$T
TAG=$T LIMIT=${LIMIT:-240} tools/r4_call.sh \
  "alone:tools/probe/shfl_probe 1 10" \
  "streams4:tools/probe/shfl_probe 4 8" \
  "beside_hog:python tools/dp_hog.py --hog 100 & H=\$!; sleep 8; tools/probe/shfl_probe 4 8; rc=\$?; kill \$H; wait \$H; exit \$rc"
