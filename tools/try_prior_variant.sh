#!/bin/bash
# Try a variant libvqa on the prior: GPU prior tests with it, then tools/bench_prior.py (train leg) base vs
# variant, twice. The product library is restored at the end. Usage: tools/try_prior_variant.sh VARIANT.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=vae-based-music--deep-generative-models_amd/libvqa.so
V=$1
cp $L gpurun_out/base.so
cp "$V" $L
timeout -k 10 400 python -u -m pytest tests/test_gpu_prior.py tests/test_gpu_sampler.py -q -x -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/variant_tests.log 2>&1
rc=$?
tail -3 gpurun_out/variant_tests.log
if [ $rc -ne 0 ]; then cp gpurun_out/base.so $L; echo "tests failed ($rc)"; exit $rc; fi
for v in gpurun_out/base.so "$V"; do
  cp "$v" $L
  echo "== seqlin shapes: $(basename $v)"
  timeout -k 10 120 python tools/seqlin_time.py || { cp gpurun_out/base.so $L; echo "seqlin_time failed"; exit 1; }
done
for r in 1 2; do
  for v in gpurun_out/base.so "$V"; do
    cp "$v" $L
    timeout -k 10 300 python tools/bench_prior.py --no-cpu --only train > gpurun_out/pb.json 2>gpurun_out/pb.err || { cp gpurun_out/base.so $L; echo "bench failed"; exit 1; }
    echo "$(basename $v) $(python -c 'import json,sys; d=json.loads(open("gpurun_out/pb.json").read().strip().splitlines()[0]); print(d["ms_per_step"], d.get("kernels"))')"
  done
done
cp gpurun_out/base.so $L
