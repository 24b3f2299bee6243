#!/bin/bash
# Round-5 GPU experiments, one runner (on the GPU box: /usr/local/graft/bin/gpurun -- 'bash tools/r5_gpu.sh NAME ...').
#   overlap            per-level exchange: RCCL / gloo parity tests, each level's end slack, world-size-1 bench A/B
#   reduce LIB...      partial-row reduction builds: per-step reduction time, then step A/B
#   fwdsm LIB...       residual-block forward builds: forward parity, per-launch sweep at short T, step A/B
#   convends LIB...    waveform-end conv builds: per-launch time, bitwise vs the product, step A/B
#   adam OLD_LIB       Keras Adam: bitwise vs OLD_LIB at two sizes, train/schedule tests, step A/B
#   close TAG          full GPU suite + smoke + round_profile.sh TAG on the in-tree library
set -o pipefail
NAME=$1; shift
OUT=gpurun_out/r5_$NAME
mkdir -p "$OUT"
case "$NAME" in
overlap)
  export HSA_ENABLE_IPC_MODE_LEGACY=0
  timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_rccl.py \
    "tests/test_gpu_dp.py::test_dp2_overlapped_exchange_bitwise_equals_one_bucket" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
  tail -8 $OUT/tests.log
  for lv in 0 1 2; do
    timeout -k 10 300 python -u tools/critpath.py --cycles 800000 --levels $lv vq_ema_apply > $OUT/slack_$lv.log 2>&1 || exit 1
    tail -2 $OUT/slack_$lv.log
  done
  for rep in 1 2; do
    for ov in 0 1; do
      VQA_DP_FORCE=1 VQA_DP_OVERLAP=$ov timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29611 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-prior \
        --no-roofline > $OUT/bench_ov${ov}_$rep.log 2>&1 || { grep -v "NCCL INFO" $OUT/bench_ov${ov}_$rep.log | head -30; exit 1; }
      grep '^{' $OUT/bench_ov${ov}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('overlap', $ov, d['ms_per_step'], d['config']['exchange'])"
    done
  done ;;
reduce)
  for v in "" "$@"; do
    echo "== reduce ${v:-product}"
    VQA_LIB_PATH=$v timeout -k 10 200 python tools/reduce_time.py 2>&1 | tail -4 || exit 1
  done
  bash tools/ab_libs.sh 2 "$@" ;;
fwdsm)
  for v in "$@"; do
    VQA_LIB_PATH=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_gpu_resblock.py -k forward > $OUT/t_$(basename $v).log 2>&1 || { tail -20 $OUT/t_$(basename $v).log; exit 1; }
    echo "$v $(tail -1 $OUT/t_$(basename $v).log)"
  done
  for v in "" "$@"; do
    echo "== sweep ${v:-product}"
    VQA_LIB_PATH=$v timeout -k 10 300 python -u tools/resblock_sweep.py --T 4096 2048 1024 512 --reps 10 2>&1 | cut -c1-60 || exit 1
  done
  bash tools/ab_libs.sh 3 "$@" ;;
convends)
  timeout -k 10 120 python tools/thin_time.py --save $OUT/prod.pt 2>&1 | grep -v amdgpu.ids || exit 1
  for v in "$@"; do
    echo "== $v"
    VQA_LIB_PATH=$v timeout -k 10 120 python tools/thin_time.py --check $OUT/prod.pt 2>&1 | grep -v amdgpu.ids || exit 1
  done
  rm -f $OUT/prod.pt  # 67 MB: gpurun_out must stay under 64 MiB to come back
  bash tools/ab_libs.sh 2 "$@" ;;
adam)
  OLD=$1
  for n in 968835 1000003; do
    VQA_LIB_PATH=$OLD timeout -k 10 120 python tools/adam_check.py --n $n --save $OUT/old_$n.pt 2>&1 | grep -v amdgpu.ids || exit 1
    timeout -k 10 120 python tools/adam_check.py --n $n --check $OUT/old_$n.pt 2>&1 | grep -v amdgpu.ids || exit 1
  done
  timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py \
    tests/test_gpu_schedule.py > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc = 0 ] || exit 1
  bash tools/ab_libs.sh 3 "$OLD" ;;
close)
  TAG=${1:-r5e}
  timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1 || exit 1
  bash tools/round_profile.sh "$TAG" > /dev/null 2>&1 || { echo "round_profile failed"; exit 1; }
  tail -5 gpurun_out/$TAG/summary.md ;;
*) echo "unknown experiment $NAME"; exit 2 ;;
esac
