# Overlapped per-level exchange: RCCL/gloo parity tests, world-size-1 bench A/B, and each level's end slack
set -o pipefail
mkdir -p gpurun_out/ovl
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_rccl.py "tests/test_gpu_dp.py::test_dp2_overlapped_exchange_bitwise_equals_one_bucket" > gpurun_out/ovl/tests.log 2>&1 || { tail -40 gpurun_out/ovl/tests.log; exit 1; }
tail -8 gpurun_out/ovl/tests.log
for lv in 0 1 2; do
timeout -k 10 300 python -u tools/critpath.py --cycles 800000 --levels $lv vq_ema_apply > gpurun_out/ovl/slack_$lv.log 2>&1 || exit 1
tail -2 gpurun_out/ovl/slack_$lv.log
done
for rep in 1 2; do
for ov in 0 1; do
VQA_DP_FORCE=1 VQA_DP_OVERLAP=$ov timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-prior --no-roofline > gpurun_out/ovl/bench_ov${ov}_$rep.log 2>&1 || { grep -v "NCCL INFO" gpurun_out/ovl/bench_ov${ov}_$rep.log | head -30; exit 1; }
grep '^{' gpurun_out/ovl/bench_ov${ov}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('overlap', $ov, d['ms_per_step'], d['config']['exchange'])"
done
done
