#!/bin/bash
# round-4 close on the shipped library: the whole -m gpu suite, smoke, the bench line, then the round profile
# (PMC traffic re-measured on this library, serialised kernel stats)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r4close tools/r4_final.sh && VQA_COMMIT=${VQA_COMMIT:-unknown} tools/round_profile.sh r4close/prof
