# Thin (1-channel) conv variants: timing, fp64 parity and bitwise equality with the product per variant
set -o pipefail
mkdir -p gpurun_out/thin
timeout -k 10 120 python tools/thin_time.py --save gpurun_out/thin/prod.pt 2>&1 | grep -v amdgpu.ids || exit 1
for v in variants/wtx.so variants/wtx16.so variants/wtx4.so variants/thinf.so variants/thinfx.so; do
  echo "== $v"
  VQA_LIB_PATH=$v timeout -k 10 120 python tools/thin_time.py --check gpurun_out/thin/prod.pt 2>&1 | grep -v amdgpu.ids || exit 1
done
VQA_LIB_PATH=variants/thinfx.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py > gpurun_out/thin/conv_tests.log 2>&1; echo "conv tests (thinfx) rc=$?"; tail -2 gpurun_out/thin/conv_tests.log
