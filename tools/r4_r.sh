#!/bin/bash
# round-4 GPU call R: spectral loss-gradient repeatability alone and with a second process on the GPU
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4r}
TAG=$T LIMIT=${LIMIT:-300} tools/r4_call.sh \
  "alone:python -u tools/spec_race.py 1 20" \
  "two:python -u tools/spec_race.py 2 20" \
  "three:python -u tools/spec_race.py 3 20"
