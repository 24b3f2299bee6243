#!/bin/bash
# round-4 GPU call H: the VQ kernels' tests first (new vectorised / rank / segment kernels), the whole -m gpu
# suite + smoke; the next change set (variants/r4dev.so: spectral gather, float4 MSE, per-item dtail grid with
# pipelined loads, 8 rows in flight in wgrad_thin) through its tests, serialised traces and the step A/B
# against the product and variants/r4base.so (the library before the EMA/quantizer change set); VQ micro
# timings; PMC passes over the residual-block backward; the argmin A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4h}
TAG=$T LIMIT=${LIMIT:-900} tools/r4_call.sh \
  "vq:python -u -m pytest tests/test_gpu_vq.py -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "all:python -u -m pytest tests -v -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider" \
  "smoke:python -c \"import __graft_entry__ as g; g.smoke()\"" \
  "dev:tools/try_lib.sh variants/r4dev.so \"tests/test_gpu_spectral.py tests/test_gpu_dtail.py tests/test_gpu_losses.py tests/test_gpu_conv.py tests/test_gpu_vq.py\" $T/dev" \
  "occ3_tests:tools/lib_tests.sh variants/r4occ3.so tests/test_gpu_resblock.py" \
  "step_ab:tools/ab_libs.sh 2 variants/r4base.so variants/r4dev.so variants/r4occ3.so" \
  "vq_ab:tools/lib_ab.sh \"python tools/vq_ema_bench.py\" variants/r4base.so" \
  "pmc_res:WHICH=both tools/pmc_res.sh $T/pmcres" \
  "argmin_ab:tools/lib_ab.sh \"python tools/argmin_time.py\" variants/argmin_old.so"
