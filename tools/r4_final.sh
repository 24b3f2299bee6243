#!/bin/bash
# round-4 final check on the committed tree: the whole -m gpu suite, smoke, the default bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4final}
TAG=$T LIMIT=${LIMIT:-900} tools/r4_call.sh \
  "all:python -u -m pytest tests -v -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider" \
  "smoke:python -c \"import __graft_entry__ as g; g.smoke()\"" \
  "bench:python bench.py"
