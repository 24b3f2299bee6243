#!/bin/bash
# A/B of variant libraries: the given GPU test files with each variant, a timing tool on base and each variant,
# and the step A/B. Usage: TESTS="tests/x.py" TOOL="python tools/t.py" tools/r3_try.sh V1.so [V2.so ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
L=vae-based-music--deep-generative-models_amd/libvqa.so
OUT=gpurun_out/r3try; mkdir -p $OUT; cp $L $OUT/base.so
for v in "$@"; do
  cp "$v" $L
  timeout -k 10 400 python -u -m pytest $TESTS -q -x -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_$(basename $v .so).log 2>&1
  rc=$?; echo "$(basename $v) tests: $(tail -1 $OUT/tests_$(basename $v .so).log)"
  cp $OUT/base.so $L
  [ $rc -ne 0 ] && exit $rc
done
for v in $OUT/base.so "$@"; do
  cp "$v" $L
  echo "== $(basename $v)"
  timeout -k 10 150 $TOOL 2>/dev/null || { cp $OUT/base.so $L; exit 1; }
done
cp $OUT/base.so $L
tools/ab_libs.sh ${ABR:-2} "$@"
