#!/bin/bash
# round-4 GPU call H: the VQ kernels' tests first (new vectorised / rank / segment kernels), the whole -m gpu
# suite + smoke, then A/Bs against variants/r4base.so (the library before this change set): VQ micro-timings,
# the step (alternating rounds), and a serialised kernel-trace of the new library
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r4h}
TAG=$T LIMIT=${LIMIT:-900} tools/r4_call.sh \
  "vq:python -u -m pytest tests/test_gpu_vq.py -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "all:python -u -m pytest tests -v -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider" \
  "smoke:python -c \"import __graft_entry__ as g; g.smoke()\"" \
  "vq_ab:tools/lib_ab.sh \"python tools/vq_ema_bench.py\" variants/r4base.so" \
  "step_ab:tools/ab_libs.sh 3 variants/r4base.so" \
  "layout_ab:tools/env_ab.sh 2 \"\" \"VQA_STEP_LAYOUT=r3\"" \
  "argmin_ab:tools/lib_ab.sh \"python tools/argmin_time.py\" variants/argmin_old.so" \
  "kstats:VQA_LEVEL_STREAMS=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/trace -o t -- python bench.py --no-cpu-baseline --no-prior --no-roofline --steps 10"
