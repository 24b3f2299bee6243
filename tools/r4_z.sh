#!/bin/bash
# round-4 GPU call Z: the DP tests (turns + measured Adam-noise bounds), the shuffle probe (alone / 4 streams /
# beside a busy process), then the round-end profile of the final library (bench line, serialised kernel stats,
# PMC traffic)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4z}
mkdir -p gpurun_out/$T
TAG=$T LIMIT=${LIMIT:-700} tools/r4_call.sh \
  "dp:python -u -m pytest tests/test_gpu_dp.py -v -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider" \
  "shfl_alone:tools/probe/shfl_probe 1 10" \
  "shfl_streams4:tools/probe/shfl_probe 4 8" \
  "shfl_beside_hog:python tools/dp_hog.py --hog 100 & H=\$!; sleep 8; tools/probe/shfl_probe 4 8; rc=\$?; kill \$H; wait \$H; exit \$rc" \
  "profile:tools/round_profile.sh $T/prof"
