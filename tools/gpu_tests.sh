#!/bin/bash
# Run GPU test files one pytest process each; stop at the first crash / timeout (exit code not 0/1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for f in "$@"; do
  timeout -k 10 ${STEP_TIMEOUT:-420} python -m pytest "$f" -m gpu -q --maxfail=${MAXFAIL:-30} -p no:cacheprovider \
    > "gpurun_out/$(basename $f .py).log" 2>&1
  rc=$?
  echo "$f exit=$rc"; tail -5 "gpurun_out/$(basename $f .py).log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $f crashed or timed out ($rc)"; exit $rc; fi
done
