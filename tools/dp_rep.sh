set -e
T="timeout -k 10 200 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_dp.py"
$T > gpurun_out/dp_full.log 2>&1
for i in 1 2 3 4; do timeout -k 10 150 python -u -m pytest -x -q --timeout 140 --timeout-method thread tests/test_gpu_dp.py -k "cfg2_short and bf16" > gpurun_out/dp_rep$i.log 2>&1; done
