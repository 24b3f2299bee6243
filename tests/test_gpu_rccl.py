"""The RCCL branch of the data-parallel exchange, executed on one GPU (SURVEY.md §8e "Collective").

Multi-GPU runs are the driver's; on a one-GPU box the product's RCCL path — `dist.init_process_group("nccl",
device_id=...)` and `dist.all_reduce` of the device bucket queued on the producer stream, then the EMA and Keras
Adam on that stream (eager) or in the second graph (captured) — runs in a world-size-1 group with
vqa_dp.FORCE_COLLECTIVE. A one-rank sum is the bucket itself, so the step must end BITWISE where the same model
without the DP path ends, eager and graph-captured. RCCL's own log (NCCL_DEBUG=INFO) must show that it ran.
bench.py's RCCL branch runs the same way: torchrun with one process and VQA_DP_FORCE=1.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rccl_env():
    return dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0", WORLD_SIZE="1",
                LOCAL_RANK="0", NCCL_DEBUG="INFO", HSA_ENABLE_IPC_MODE_LEGACY="0")


def _rccl_lines(text):
    return [ln for ln in text.splitlines() if "NCCL INFO" in ln or "RCCL" in ln]


@pytest.mark.timeout(600)
def test_rccl_world1_step_equals_single_process_bitwise(cuda, tmp_path):
    out = str(tmp_path / "rccl.pt")
    p = subprocess.run([sys.executable, os.path.join(HERE, "rccl_worker.py"), out], env=_rccl_env(),
                       capture_output=True, text=True, timeout=540)
    log = p.stdout + p.stderr
    assert p.returncode == 0, log[-4000:]
    lines = _rccl_lines(log)
    print("\n".join(lines[:12]))
    assert lines, "no RCCL log line (NCCL_DEBUG=INFO): the nccl backend did not run"
    res = torch.load(out, weights_only=True)
    for mode in ("eager", "graph"):
        dp, single = res[f"{mode}_dp"], res[f"{mode}_single"]
        calls = dp["all_reduce_calls"]
        # eager: one exchange per step; graph: the warm-up step's and each replay's exchange
        assert len(calls) == (2 if mode == "eager" else 3), calls
        assert all(c["backend"] == "nccl" and c["device"].startswith("cuda") and c["numel"] == dp["grads"].numel()
                   + dp["stats"].numel() for c in calls), calls
        assert not single["all_reduce_calls"], "the single-process path runs no collective"
        for k in ("weights", "adam_m", "adam_v", "grads", "stats"):
            n = int((dp[k] != single[k]).sum())
            assert n == 0, f"{mode}: {k} differs in {n} elements between the RCCL path and the single-process step"
        for a, b in zip(dp["vq"], single["vq"]):
            assert a["calls"] == b["calls"]
            for k in ("embeddings", "m_t", "N_t"):
                assert torch.equal(a[k], b[k]), f"{mode}: codebook {k} differs"
        assert dp["results"] == single["results"], f"{mode}: metrics differ"


@pytest.mark.timeout(600)
def test_rccl_world1_overlapped_exchange_equals_single_process_bitwise(cuda, tmp_path):
    """VQVAE.overlap_exchange on the RCCL branch: per step one ncclAllReduce per level region (gradient range, VQ
    statistics), issued straight to the process group's communicator on the exchange stream right after that
    level's backward, then the losses after the join; in graph mode the collectives are CAPTURED with the step
    into one hipGraph (no split graphs). One rank: bitwise the single-process step, eager and graph."""
    out = str(tmp_path / "rccl_ovl.pt")
    p = subprocess.run([sys.executable, os.path.join(HERE, "rccl_worker.py"), out, "overlap"], env=_rccl_env(),
                       capture_output=True, text=True, timeout=540)
    log = p.stdout + p.stderr
    assert p.returncode == 0, log[-4000:]
    assert _rccl_lines(log), "no RCCL log line (NCCL_DEBUG=INFO): the nccl backend did not run"
    res = torch.load(out, weights_only=True)
    for mode in ("eager", "graph"):
        dp, single = res[f"{mode}_dp"], res[f"{mode}_single"]
        regs = dp["regions"]
        sizes = [b - a for lv in regs[:-1] for a, b in lv] + [regs[-1][1] - regs[-1][0]]
        # ncclAllReduce issued directly on the process group's communicator (vqa_dp._Rccl; at most the one
        # torch collective that creates a lazily built communicator goes through torch.distributed);
        # eager: two steps; graph: the warm-up step and the capture (replays re-issue nothing from the host)
        calls = dp["direct_calls"]
        assert len(dp["all_reduce_calls"]) <= 1, dp["all_reduce_calls"]
        assert sorted(calls) == sorted(sizes * 2), calls
        assert not single["all_reduce_calls"] and not single["direct_calls"]
        for k in ("weights", "adam_m", "adam_v", "grads", "stats"):
            n = int((dp[k] != single[k]).sum())
            assert n == 0, f"{mode}: {k} differs in {n} elements between the overlapped RCCL path and the single step"
        for a, b in zip(dp["vq"], single["vq"]):
            assert a["calls"] == b["calls"]
            for k in ("embeddings", "m_t", "N_t"):
                assert torch.equal(a[k], b[k]), f"{mode}: codebook {k} differs"
        assert dp["results"] == single["results"], f"{mode}: metrics differ"


@pytest.mark.timeout(600)
@pytest.mark.parametrize("overlap", ["0", "1"])
def test_bench_py_rccl_branch_one_process(cuda, overlap):
    """bench.py under torch.distributed.run with one process and VQA_DP_FORCE=1: init_process_group("nccl",
    device_id=...), the split-graph DP step with an RCCL all_reduce per step, barrier + max-over-ranks timing."""
    env = _rccl_env()
    env.update(VQA_DP_FORCE="1", OMP_NUM_THREADS="4", VQA_DP_OVERLAP=overlap)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "3",
           "--warmup", "2", "--batch", "2", "--seq", "8192", "--no-cpu-baseline", "--no-prior", "--no-fp32", "--no-roofline"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=540, cwd=ROOT)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    assert _rccl_lines(p.stdout + p.stderr), "no RCCL log line from bench.py's process group"
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["config"]["parallelism"] == "dp1" and out["value"] > 0
    assert out["config"]["exchange"] == ("per-level, overlapped" if overlap == "1" else "one bucket after the join")
