#!/bin/bash
# Round-6 GPU experiments, one runner (on the GPU box: /usr/local/graft/bin/gpurun -- 'bash tools/r6_gpu.sh NAME ...').
#   entry              the round's new GPU tests (bare bench --gpus 2, replay after test_step, random-delay race),
#                      the RCCL world-size-1 tests, then ONE capture probe form (argument; may segfault: last step)
#   probe FORM         tools/capture_fork_probe.py FORM alone (world size 1)
#   rsab LIB...        residual-block builds: outputs bitwise vs variants/libvqa_r5.so (tools/rs_bitwise.py),
#                      tests/test_gpu_resblock.py, per-launch sweep (r5 and each build), step A/B (in-tree vs builds)
#   stamps LIB...      per-phase s_memtime stamps (libraries built with -DVQA_RS_STAMPS): backward d = 1, 9, 27 and
#                      the forward, T = 32768
#   spec LIB...        spectral builds: tests, per-kernel averages, graph-timed target + loss/grad, step A/B
#   rsweep LIB...      per-launch residual-block sweep, r5 and each build
#   sweepab LIB...     per-launch sweep of each build, then the step A/B (in-tree library as the base)
#   dtab LIB...        decoder-tail builds: tests, launch times + digests, per-kernel averages, step A/B
#   convab LIB...      waveform-end conv builds: conv tests, first-conv times + digests, per-kernel averages, step A/B
#   sweeps LIB...      per-shape conv sweep of the in-tree library and each build, then the step A/B (ROUNDS)
#   priorab LIB...     prior builds: prior tests, then the config-4 train step alternating with the in-tree library
#   suite              full GPU suite + smoke + the default bench line (in-tree library)
#   close TAG          (VQA_COMMIT=<head>) full GPU suite + smoke + round_profile.sh TAG on the in-tree library
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
rsab)
  VQA_LIB_PATH=variants/libvqa_r5.so timeout -k 10 300 python -u tools/rs_bitwise.py --save $OUT/ref.pt 2>&1 \
    | grep -v amdgpu.ids || exit 1
  for v in "$@"; do
    echo "== bitwise $v"
    VQA_LIB_PATH=$v timeout -k 10 300 python -u tools/rs_bitwise.py --check $OUT/ref.pt 2>&1 | grep -v amdgpu.ids | tail -40
    [ ${PIPESTATUS[0]} -le 1 ] || exit 1
  done
  rm -f $OUT/ref.pt
  for v in "$@"; do
    VQA_LIB_PATH=$v timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
      tests/test_gpu_resblock.py > $OUT/t_$(basename $v).log 2>&1 || { tail -30 $OUT/t_$(basename $v).log; exit 1; }
    echo "tests $v: $(tail -1 $OUT/t_$(basename $v).log)"
  done
  for v in variants/libvqa_r5.so "$@"; do
    echo "== sweep $v"
    VQA_LIB_PATH=$v timeout -k 10 300 python -u tools/resblock_sweep.py --T 32768 8192 2048 512 --reps 10 --fused-only 2>&1 \
      | grep -v amdgpu.ids || exit 1
  done
  bash tools/ab_libs.sh 3 variants/libvqa_r5.so "$@" ;;
stamps)
  for v in "$@"; do
    echo "== stamps $v"
    VQA_LIB_PATH=$v timeout -k 10 300 python -u tools/rs_stamps.py --T 32768 --d 1 9 27 2>&1 | grep -v amdgpu.ids || exit 1
    VQA_LIB_PATH=$v timeout -k 10 300 python -u tools/rs_stamps.py --T 32768 --d 1 9 27 --fwd 2>&1 | grep -v amdgpu.ids || exit 1
  done ;;
spec)
  # spectral builds: tests/test_gpu_spectral.py on each, per-kernel averages (rocprofv3 --stats over tools/spec_one.py)
  # and the graph-timed target + loss/grad for the r5 library and each build, then the step A/B
  export TMPDIR=/tmp
  for v in "$@"; do
    VQA_LIB_PATH=$v timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
      tests/test_gpu_spectral.py > $OUT/t_$(basename $v).log 2>&1 || { tail -40 $OUT/t_$(basename $v).log; exit 1; }
    echo "tests $v: $(tail -1 $OUT/t_$(basename $v).log)"
  done
  for v in ${SPEC_BASE:-variants/libvqa_r5.so} "$@"; do
    n=$(basename $v .so)
    VQA_LIB_PATH=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o t -- \
      python tools/spec_one.py 5 > /dev/null 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }
    echo "== $v: $(VQA_LIB_PATH=$v timeout -k 10 120 python tools/spec_one.py --time 2>/dev/null | head -1)"
    python - "$OUT/$n/t_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "spec" in r["Name"]:
        print(f"   {r['Name'][:60]:60s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
    find $OUT/$n -name "*kernel_trace.csv" -delete
  done
  bash tools/ab_libs.sh 3 ${SPEC_BASE:-variants/libvqa_r5.so} "$@" ;;
rsweep)
  # per-launch residual-block times only (tools/resblock_sweep.py --fused-only), the r5 library and each build
  for v in variants/libvqa_r5.so "$@"; do
    echo "== sweep $v"
    VQA_LIB_PATH=$v timeout -k 10 300 python -u tools/resblock_sweep.py --T 32768 8192 2048 512 --reps 10 --fused-only 2>&1 \
      | grep -v amdgpu.ids || exit 1
  done ;;
sweepab)
  # per-launch residual-block sweep for each build, then the step A/B against the in-tree library
  for v in "$@"; do
    echo "== sweep $v"
    VQA_LIB_PATH=$v timeout -k 10 300 python -u tools/resblock_sweep.py --T 32768 8192 4096 2048 512 --reps 10 --fused-only \
      2>&1 | grep -v amdgpu.ids || exit 1
  done
  bash tools/ab_libs.sh 3 "$@" ;;
dtab)
  # decoder-tail builds: tests/test_gpu_dtail.py, launch times + digest (tools/dtail_one.py), per-kernel averages,
  # then the step A/B against the in-tree library
  export TMPDIR=/tmp
  for v in "$@"; do
    VQA_LIB_PATH=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_gpu_dtail.py > $OUT/t_$(basename $v).log 2>&1 || { tail -40 $OUT/t_$(basename $v).log; exit 1; }
    echo "tests $v: $(tail -1 $OUT/t_$(basename $v).log)"
  done
  for v in vae-based-music--deep-generative-models_amd/libvqa.so "$@"; do
    n=$(basename $v .so)
    echo "== $v"
    VQA_LIB_PATH=$v timeout -k 10 120 python -u tools/dtail_one.py 2>&1 | grep -v amdgpu.ids || exit 1
    VQA_LIB_PATH=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o t -- \
      python tools/dtail_one.py > /dev/null 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }
    python - "$OUT/$n/t_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"   {r['Name'][:60]:60s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
    find $OUT/$n -name "*kernel_trace.csv" -delete
  done
  bash tools/ab_libs.sh 3 "$@" ;;
convab)
  # waveform-end conv builds: tests/test_gpu_conv.py on each, the first conv's forward / weight-gradient times and
  # output digest (tools/first_conv.py) for the in-tree library and each build, per-kernel averages, step A/B
  export TMPDIR=/tmp
  for v in "$@"; do
    VQA_LIB_PATH=$v timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
      tests/test_gpu_conv.py > $OUT/t_$(basename $v).log 2>&1 || { tail -40 $OUT/t_$(basename $v).log; exit 1; }
    echo "tests $v: $(tail -1 $OUT/t_$(basename $v).log)"
  done
  for v in vae-based-music--deep-generative-models_amd/libvqa.so "$@"; do
    n=$(basename $v .so)
    echo "== $v"
    VQA_LIB_PATH=$v timeout -k 10 120 python -u tools/first_conv.py 2>&1 | grep -v amdgpu.ids || exit 1
    VQA_LIB_PATH=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o t -- \
      python tools/first_conv.py > /dev/null 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }
    python - "$OUT/$n/t_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "vqa" in r["Name"]:
        print(f"   {r['Name'][:60]:60s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
    find $OUT/$n -name "*kernel_trace.csv" -delete
  done
  bash tools/ab_libs.sh 3 "$@" ;;
sweeps)
  # per-shape conv times of one eager step (tools/conv_sweep.py) for the in-tree library and each build, then the
  # step A/B (ROUNDS rounds; env, default 3)
  for v in vae-based-music--deep-generative-models_amd/libvqa.so "$@"; do
    echo "== conv sweep $v"
    VQA_LIB_PATH=$v timeout -k 10 300 python -u tools/conv_sweep.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
  bash tools/ab_libs.sh ${ROUNDS:-3} "$@" ;;
priorab)
  # prior builds: tests/test_gpu_prior.py on each, then the config-4 train step (tools/bench_prior.py --only train)
  # alternating the in-tree library and each build (ROUNDS, default 3)
  for v in "$@"; do
    VQA_LIB_PATH=$v timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
      tests/test_gpu_prior.py > $OUT/t_$(basename $v).log 2>&1 || { tail -40 $OUT/t_$(basename $v).log; exit 1; }
    echo "tests $v: $(tail -1 $OUT/t_$(basename $v).log)"
  done
  for r in $(seq ${ROUNDS:-3}); do
    for v in vae-based-music--deep-generative-models_amd/libvqa.so "$@"; do
      echo "$(basename $v) $(VQA_LIB_PATH=$v timeout -k 10 300 python tools/bench_prior.py --only train --no-cpu 2>/dev/null | tail -1)"
    done
  done ;;
suite)
  timeout -k 10 2400 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/suite.log 2>&1 \
    || { tail -60 $OUT/suite.log; exit 1; }
  tail -3 $OUT/suite.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2 || exit 1
  timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['value'], d['roofline']['avg_launch_us'], {k: (v.get('ms_per_step'), v.get('value')) for k, v in d.items() if k.startswith('config')})" ;;
close)
  [ -n "$VQA_COMMIT" ] || { echo "close: set VQA_COMMIT (the git HEAD sent)"; exit 2; }
  TAG=$1
  timeout -k 10 2400 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/suite.log 2>&1 \
    || { tail -60 $OUT/suite.log; exit 1; }
  tail -3 $OUT/suite.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2 || exit 1
  bash tools/round_profile.sh "$TAG" ;;
*)
  echo "unknown experiment $NAME"; exit 2 ;;
esac
