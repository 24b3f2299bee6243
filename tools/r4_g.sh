#!/bin/bash
# round-4 GPU call: the whole -m gpu suite + smoke (the driver's round-end tiers), step-layout and argmin A/B,
# spectral PMC passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r4g} LIMIT=${LIMIT:-900} tools/r4_call.sh \
  "all:python -u -m pytest tests -v -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider" \
  "smoke:python -c \"import __graft_entry__ as g; g.smoke()\"" \
  "layout_ab:tools/env_ab.sh 2 \"\" \"VQA_STEP_LAYOUT=r3\"" \
  "argmin_ab:tools/lib_ab.sh \"python tools/argmin_time.py\" variants/argmin_old.so" \
  "spec_pmc:tools/pmc_kernel.sh ${TAG:-r4g}/spec_pmc spec_pair_kernel -- python tools/spec_one.py 3"
