"""The product's data-parallel step: two ranks (gloo, both on cuda:0) drive VQVAE with a
process group — eager, and graph-captured (two hipGraphs around the eager all_reduce) — and must end where
a single process training on the concatenated global batch ends: code counts bitwise, the same global reset rows,
EMA sums / codebooks / weights / Adam moments within fp32 rounding of the different summation grouping
(rank-local sums then the all_reduce), metrics alike; both ranks identical to each other bitwise. Then one
forward-only `vqvaes[0](x, training=True)` (the EMA on the global batch's statistics) likewise.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import dp_worker as W  # noqa: E402

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(mode, tmp_path, world=2):
    port = _port()
    procs, outs = [], []
    for r in range(world):
        out = str(tmp_path / f"{mode}_rank{r}.pt")
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dp_worker.py"), mode, out], env=env))
        outs.append(out)
    for p in procs:
        assert p.wait(timeout=300) == 0
    return [torch.load(o, weights_only=True) for o in outs]


def _single(world=2):
    m = W.build(W.B_LOCAL * world)
    xs = W.batches(world)
    m.train_step(xs[0])
    m.train_step(xs[1])
    torch.cuda.synchronize()
    res = {"steps": W.snapshot(m)}
    m.vqvaes[0](xs[2], training=True)
    torch.cuda.synchronize()
    res["forward"] = W.snapshot(m)
    return res


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


@pytest.mark.parametrize("mode", ["eager", "graph"])
def test_dp2_matches_single_process_global_batch(cuda, tmp_path, mode):
    ranks = _run_ranks(mode, tmp_path)
    ref = _single()
    K, D = W.CFG["num_embeddings"], W.CFG["latent_dim"]
    assert torch.equal(ranks[0]["steps"]["stats"], ranks[1]["steps"]["stats"])  # incl. the exchanged losses
    for phase in ("steps", "forward"):
        r0, r1, s = ranks[0][phase], ranks[1][phase], ref[phase]
        # replicas identical (the EMA statistics; after the forward-only call the loss slots hold each rank's
        # local commitment loss, as vqvaes[l].losses does in the reference)
        nst = 2 * K * D + K
        assert torch.equal(r0["weights"], r1["weights"]) and torch.equal(r0["stats"][:nst], r1["stats"][:nst])
        for a, b in zip(r0["vq"], r1["vq"]):
            assert all(torch.equal(a[k], b[k]) for k in ("embeddings", "m_t", "N_t")) and a["calls"] == b["calls"]
        # vs one process on the global batch
        st, ss = r0["stats"], s["stats"]
        m_sum, n_sum, RT = st[:K * D], st[K * D:K * D + K], st[K * D + K:2 * K * D + K]
        assert torch.equal(n_sum, ss[K * D:K * D + K]), f"{phase}: code counts"
        # the same global rows selected (their values carry step 1's fp32 weight differences)
        assert _rel(RT, ss[K * D + K:2 * K * D + K]) < 1e-5, f"{phase}: reset rows"
        assert _rel(m_sum, ss[:K * D]) < 1e-6, f"{phase}: EMA sums"
        if phase == "steps":
            # the exchanged gradient (sum over ranks of rank-mean gradients) = world x the global-batch mean
            # gradient, to fp32 rounding of the different summation grouping
            assert _rel(r0["grads"] / 2, s["grads"]) < 2e-6, f"{phase}: gradients"
        # Adam normalises each element by sqrt(v): an element whose gradient nearly cancels across items keeps
        # its absolute rounding noise but has a small sqrt(v), so a 1e-7-relative gradient difference becomes
        # up to ~1e-3 of that element's update (Keras default lr = 1e-3 per step), i.e. a few 1e-6 of max|w|
        assert _rel(r0["weights"], s["weights"]) < 1e-5, f"{phase}: weights"
        if phase == "steps":
            assert _rel(r0["adam_m"], s["adam_m"]) < 1e-5 and _rel(r0["adam_v"], s["adam_v"]) < 1e-5
        for a, b in zip(r0["vq"], s["vq"]):
            assert torch.equal(a["N_t"], b["N_t"]) and a["calls"] == b["calls"]
            assert _rel(a["embeddings"], b["embeddings"]) < 1e-5 and _rel(a["m_t"], b["m_t"]) < 1e-5
        for k, v in s["results"].items():
            assert abs(r0["results"][k] - v) <= 1e-5 * max(abs(v), 1e-3), f"{phase} {k}: {r0['results'][k]} vs {v}"
