#!/bin/bash
# Per-shape sequence-linear timings (tools/seqlin_time.py) for the product library and variant builds, after the
# prior GPU tests pass with each variant. The product library is restored at the end.
# Usage: tools/ab_seqlin.sh VARIANT.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=vae-based-music--deep-generative-models_amd/libvqa.so
cp $L gpurun_out/base.so
for v in "$@"; do
  cp "$v" $L
  timeout -k 10 300 python -u -m pytest tests/test_gpu_prior.py -q -x -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/variant_tests.log 2>&1 || { cp gpurun_out/base.so $L; echo "tests failed for $v"; tail -20 gpurun_out/variant_tests.log; exit 1; }
  echo "$(basename $v): $(tail -1 gpurun_out/variant_tests.log)"
done
for v in gpurun_out/base.so "$@"; do
  cp "$v" $L
  echo "== $(basename $v)"
  timeout -k 10 120 python tools/seqlin_time.py | cut -c1-60 || { cp gpurun_out/base.so $L; echo "seqlin_time failed"; exit 1; }
done
cp gpurun_out/base.so $L
