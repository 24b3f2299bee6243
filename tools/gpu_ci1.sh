# First encoder conv forward variants: per-launch time + bitwise vs product, then step A/B
set -o pipefail
mkdir -p gpurun_out/ci1
timeout -k 10 120 python tools/thin_time.py --save gpurun_out/ci1/prod.pt 2>&1 | grep -v amdgpu.ids | head -1 || exit 1
for v in "$@"; do
  echo "== $v"
  VQA_LIB_PATH=$v timeout -k 10 120 python tools/thin_time.py --check gpurun_out/ci1/prod.pt 2>&1 | grep -v amdgpu.ids | grep -v "rel err" || exit 1
done
rm -f gpurun_out/ci1/prod.pt
bash tools/ab_libs.sh 2 "$@"
