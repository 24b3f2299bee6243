# Vectorised Keras Adam: bitwise vs the previous build, per-launch time, step A/B
set -o pipefail
mkdir -p gpurun_out/adam
VQA_LIB_PATH=variants/old.so timeout -k 10 120 python tools/adam_check.py --save gpurun_out/adam/old.pt 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 python tools/adam_check.py --check gpurun_out/adam/old.pt 2>&1 | grep -v amdgpu.ids || exit 1
VQA_LIB_PATH=variants/old.so timeout -k 10 120 python tools/adam_check.py --n 1000003 --save gpurun_out/adam/old3.pt 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 python tools/adam_check.py --n 1000003 --check gpurun_out/adam/old3.pt 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_schedule.py > gpurun_out/adam/tests.log 2>&1; rc=$?; tail -2 gpurun_out/adam/tests.log; [ $rc = 0 ] || exit 1
bash tools/ab_libs.sh 3 variants/old.so
