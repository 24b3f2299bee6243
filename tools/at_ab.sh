#!/bin/bash
# Prior attention variant on the GPU box: test_gpu_prior with it, then tools/bench_prior.py (train leg) for the
# product library and the variant. Usage: tools/at_ab.sh VARIANT.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=vae-based-music--deep-generative-models_amd/libvqa.so
OUT=gpurun_out/at_ab
mkdir -p $OUT
cp $L $OUT/base.so
cp "$1" $L
timeout -k 10 300 python -u -m pytest tests/test_gpu_prior.py tests/test_gpu_sampler.py -q -x -m gpu --timeout 250 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "variant tests: $(tail -1 $OUT/tests.log)"
cp $OUT/base.so $L
[ $rc -ne 0 ] && exit $rc
for v in $OUT/base.so "$1"; do
  cp "$v" $L
  echo "== $(basename $v)"; timeout -k 10 300 python tools/bench_prior.py --no-cpu --only train 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d.get("kernels"))'
done
cp $OUT/base.so $L
