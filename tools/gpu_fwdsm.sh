# Forward residual block with smaller tiles for short items: parity per variant, per-launch sweep, step A/B
set -o pipefail
mkdir -p gpurun_out/fwdsm
for v in fwdsm128 fwdsm96 fwdsm64; do
  VQA_LIB_PATH=variants/$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_resblock.py -k forward > gpurun_out/fwdsm/t_$v.log 2>&1 || { tail -20 gpurun_out/fwdsm/t_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/fwdsm/t_$v.log)"
done
for v in "" variants/fwdsm128.so variants/fwdsm96.so variants/fwdsm64.so; do
  echo "== sweep ${v:-product}"
  VQA_LIB_PATH=$v timeout -k 10 300 python -u tools/resblock_sweep.py --T 4096 2048 1024 512 --reps 10 2>&1 | cut -c1-60 || exit 1
done
bash tools/ab_libs.sh 3 variants/fwdsm128.so variants/fwdsm96.so
