# Thin (1-channel) conv variants: timing, fp64 parity and bitwise equality with the product per variant
set -o pipefail
mkdir -p gpurun_out/thin
timeout -k 10 120 python tools/thin_time.py --save gpurun_out/thin/prod.pt 2>&1 | grep -v amdgpu.ids || exit 1
for v in "$@"; do
  echo "== $v"
  VQA_LIB_PATH=$v timeout -k 10 120 python tools/thin_time.py --check gpurun_out/thin/prod.pt 2>&1 | grep -v amdgpu.ids || exit 1
done
