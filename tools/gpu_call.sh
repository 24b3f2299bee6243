#!/bin/bash
# One GPU call: steps given as "name:command" words; each runs under its own time limit. A step that
# fails its assertions (exit 1) lets the next one run; a time limit, abort or fault (any other non-zero status)
# ends the script there.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-call}
mkdir -p "$OUT"
export TMPDIR=/tmp
LIMIT=${LIMIT:-600}
status=0
for step in "$@"; do
  name=${step%%:*}
  cmd=${step#*:}
  echo "== $name: $cmd" | tee -a "$OUT/steps.txt"
  timeout -k 10 "$LIMIT" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "   rc=$rc $(tail -1 "$OUT/$name.log" | cut -c1-200)" | tee -a "$OUT/steps.txt"
  if [ $rc -ne 0 ]; then
    status=1
    if [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  fi
done
exit $status
