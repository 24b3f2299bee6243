"""The prior's data-parallel step (BASELINE config 4 is 8-GPU DP): two ranks (gloo, both on cuda:0) drive
Prior.train_step with a process group — eager and as two hipGraphs around the eager all_reduce — and must end
where one process training on the concatenated batch ends: the teacher-forcing draw over global rows
identical, loss / accuracy trackers equal, the exchanged gradients = 2 x the global-batch mean gradient (fp32
rounding of the grouping), weights after Keras Adam within Adam's per-element amplification, replicas
bitwise identical. With dropout 0.1 (the reference default) the masks are keyed on the global element index,
so the ranks apply the single-process masks of the global batch and the same bounds hold.
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import prior_dp_worker as W  # noqa: E402

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


@pytest.mark.parametrize("mode", ["eager", "graph", "eager_cond", "graph_cond", "eager_drop", "graph_cond_drop",
                                  "eager_full", "graph_full"])
def test_prior_dp2_matches_single_process(cuda, tmp_path, mode, monkeypatch):
    """`_full`: BASELINE config 4's SMALL_PRIOR at its own size (ctx 8192, 2048 bins, depth 6), one sequence per
    rank against one process on both, within the same bounds as the short form."""
    port = _port()
    full = mode.endswith("_full")
    mode = mode.replace("_full", "")
    monkeypatch.setenv("VQA_PRIOR_DP_FULL", "1" if full else "0")
    procs, outs = [], []
    for r in range(2):
        out = str(tmp_path / f"{mode}_rank{r}.pt")
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "prior_dp_worker.py"), mode, out], env=env))
        outs.append(out)
    for p in procs:
        assert p.wait(timeout=300) == 0
    r0, r1 = (torch.load(o, weights_only=True) for o in outs)
    cond = "_cond" in mode  # the upsampler form: ConditionerNet on upper-level codes + genre labels
    single = W.build(cond=cond, drop="_drop" in mode)
    xs = [W.to_dev(x) for x in W.batches(2, cond)]
    single.train_step(xs[0])
    single.train_step(xs[1])
    torch.cuda.synchronize()
    s = W.snapshot(single)
    assert torch.equal(r0["weights"], r1["weights"]) and torch.equal(r0["grads"], r1["grads"])
    # the same global teacher-forcing rows: each rank's mixed input is its shard of the single-process one
    assert torch.equal(torch.cat([r0["batch_input"], r1["batch_input"]]), s["batch_input"])
    assert abs(r0["loss"] - s["loss"]) <= 1e-5 * abs(s["loss"])
    assert abs(r0["accuracy"] - s["accuracy"]) <= 1e-6
    assert _rel(r0["grads"] / 2, s["grads"]) < 2e-5
    assert _rel(r0["weights"], s["weights"]) < 1e-5
