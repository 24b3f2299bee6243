# Round-5 late check: full GPU suite + smoke + bench on the product library, then reduce-kernel variants
set -o pipefail
mkdir -p gpurun_out/r5d
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/r5d/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r5d/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r5d/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r5d/bench.json 2> gpurun_out/r5d/bench.err || exit 1
cut -c1-200 gpurun_out/r5d/bench.json
for v in "" variants/red16.so variants/red16nt.so variants/red4.so; do
  echo "== reduce ${v:-product}"
  VQA_LIB_PATH=$v timeout -k 10 200 python tools/reduce_time.py 2>&1 | tail -4 || exit 1
done
bash tools/ab_libs.sh 2 variants/red16.so variants/red16nt.so
