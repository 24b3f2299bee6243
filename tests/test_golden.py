"""The oracle against its committed golden fixtures (tests/golden/, written by make_golden.py).

Since the reference cannot run here (TensorFlow absent, no fixtures of its own), these freeze the
KAT-pinned restatement: any drift in the oracle's semantics fails here before it can move the GPU
parity targets."""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as G  # noqa: E402

GOLD = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def micro_run():
    return G.run(G.MICRO, 2, 2, 100)


def test_micro_fixture_inputs_and_init(micro_run):
    cfg, params, vq, out, w, vqs = micro_run
    z = np.load(os.path.join(GOLD, "micro.npz"))
    for s in range(2):
        assert np.array_equal(z[f"x{s}"], out["x"][s])
    for n, v in params.items():
        assert np.array_equal(z[f"init/{n}"], v)
    for l, st in enumerate(vq):
        assert np.array_equal(z[f"vq_init{l}/embeddings"], st["embeddings"])


def test_micro_fixture_step_outputs(micro_run):
    cfg, params, vq, out, w, vqs = micro_run
    z = np.load(os.path.join(GOLD, "micro.npz"))
    meta = json.load(open(os.path.join(GOLD, "micro.json")))
    for s in range(2):
        for k, v in meta["metrics"][s].items():
            assert abs(out["metrics"][s][k] - v) <= 1e-10 * max(1.0, abs(v)), (s, k)
        for l in range(cfg.levels):
            assert np.array_equal(z[f"idx{s}_l{l}"], out["idx"][s][l])
        for n, g in out["grads"][s].items():
            assert np.allclose(z[f"grad{s}/{n}"], g, rtol=1e-9, atol=1e-14), (s, n)
    for n, v in w.items():
        assert np.allclose(z[f"final/{n}"], v, rtol=1e-9, atol=1e-12), n
    for l, st in enumerate(vqs):
        for k in ("embeddings", "m_t", "N_t"):
            assert np.allclose(z[f"vq_final{l}/{k}"], st[k], rtol=1e-9, atol=1e-12), (l, k)


def test_cfg1_fixture_step_scalars():
    meta = json.load(open(os.path.join(GOLD, "cfg1.json")))
    cfg, params, vq, out, w, vqs = G.run(meta["config"], meta["batch"], 1, meta["x_seeds"][0])
    for k, v in meta["metrics"][0].items():
        assert abs(out["metrics"][0][k] - v) <= 1e-10 * max(1.0, abs(v)), k
    for n, g in out["grads"][0].items():
        assert abs(np.linalg.norm(g) - meta["grad_norms"][0][n]) <= 1e-9 * meta["grad_norms"][0][n], n
