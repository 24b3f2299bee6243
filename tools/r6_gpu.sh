#!/bin/bash
# Round-6 GPU experiments, one runner (on the GPU box: /usr/local/graft/bin/gpurun -- 'bash tools/r6_gpu.sh NAME ...').
#   entry              the round's new GPU tests (bare bench --gpus 2, replay after test_step, random-delay race),
#                      the RCCL world-size-1 tests, then ONE capture probe form (argument; may segfault: last step)
#   probe FORM         tools/capture_fork_probe.py FORM alone (world size 1)
#   close TAG          full GPU suite + smoke + round_profile.sh TAG on the in-tree library
set -o pipefail
NAME=$1; shift
OUT=gpurun_out/r6_$NAME
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
probe() {
  MASTER_ADDR=127.0.0.1 MASTER_PORT=29633 timeout -k 10 120 python -u tools/capture_fork_probe.py "$1" > $OUT/probe_$1.log 2>&1
  rc=$?
  echo "probe $1 rc=$rc"; grep -v "NCCL INFO" $OUT/probe_$1.log | tail -25
  return $rc
}
case "$NAME" in
entry)
  timeout -k 10 1200 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
    "tests/test_gpu_dp.py::test_bench_py_bare_gpus2_spawns_ranks" \
    "tests/test_gpu_dp.py::test_dp2_graph_replay_after_eager_test_step_overlapped" \
    tests/test_gpu_race.py tests/test_gpu_rccl.py > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
  grep -E "PASSED|FAILED|passed|failed" $OUT/tests.log | tail -12
  [ -n "$1" ] && probe "$1" ;;
probe)
  probe "$1" ;;
close)
  TAG=$1
  timeout -k 10 2400 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/suite.log 2>&1 \
    || { tail -60 $OUT/suite.log; exit 1; }
  tail -3 $OUT/suite.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2 || exit 1
  bash tools/round_profile.sh "$TAG" ;;
*)
  echo "unknown experiment $NAME"; exit 2 ;;
esac
