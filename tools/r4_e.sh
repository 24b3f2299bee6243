#!/bin/bash
# round-4 GPU call: new kernels' parity, spectral / argmin / reduce A/B, step profile, DP checks
cd "${GRAFT_REPO_ROOT:-/root/repo}"
B="python -u bench.py --no-cpu-baseline --no-prior --steps 20"
TAG=${TAG:-r4e} LIMIT=${LIMIT:-600} tools/r4_call.sh \
  "tests:python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_vq.py tests/test_gpu_train.py -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -x" \
  "spec_prof:tools/spec_prof.sh" \
  "argmin_ab:tools/lib_ab.sh \"python tools/argmin_time.py\" variants/argmin_old.so" \
  "step_ab:tools/lib_ab.sh \"$B\" variants/reduce_old.so variants/argmin_old.so" \
  "step_prof:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG:-r4e}/prof -o t -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-prior --no-roofline" \
  "gloo_probe:python -u tools/gloo_stream_probe.py" \
  "dp:python -u -m pytest tests/test_gpu_dp.py -v -m gpu --timeout 900 --timeout-method thread -p no:cacheprovider -k config3" \
  "olddp1:VQA_DP_GLOO_DEVICE=1 python -u -m pytest tests/test_gpu_dp.py -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -k cfg2_short-bf16-graph" \
  "olddp2:VQA_DP_GLOO_DEVICE=1 python -u -m pytest tests/test_gpu_dp.py -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -k cfg2_short-bf16-graph"
