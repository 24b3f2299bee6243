"""Generate the golden fixtures from the CPU oracle (fp64). TEST INFRASTRUCTURE.

The reference (TensorFlow 2.7) cannot be imported in this container and ships no fixtures of its own, so
these vectors freeze the oracle's restatement (pinned by tests/test_oracle_kat.py) and give the GPU tests
a stored target. Re-run only when the oracle's semantics are deliberately changed:
    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import vqvae_ref as R  # noqa: E402

MICRO = dict(input_len=2048, levels=2, latent_dim=4, down_depth=[2, 1], strides=[2, 2], num_embeddings=64,
             residual_width=8, residual_depth=2, dilation_factor=3)
CFG1 = dict(input_len=4096, levels=1, latent_dim=64, down_depth=[3], strides=[2], num_embeddings=256,
            residual_width=32, residual_depth=4, dilation_factor=3)


def _rel_margin(dist):
    """(second-smallest - smallest) / |smallest| of each row's fp64 distances: how far the row is from a tie."""
    top2 = torch.topk(dist, 2, dim=1, largest=False).values
    return ((top2[:, 1] - top2[:, 0]) / top2[:, 0].abs().clamp(min=1e-30)).numpy()


def run(cfgd, B, steps, seed_x):
    cfg = R.RefConfig(**cfgd)
    params, vq = R.init_params(cfg, 1), R.init_vq_state(cfg, 2)
    m = R.RefVQVAE(cfg, params, vq, dtype=torch.float64)
    out = {"x": [], "metrics": [], "grads": [], "idx": []}
    for s in range(steps):
        x = R.synthetic_batch(B, cfg.input_len, seed=seed_x + s)
        out["x"].append(x)
        out["metrics"].append(m.train_step(x))
        out["grads"].append({n: g.numpy().astype(np.float64) for n, g in m.last["grads"].items()})
        out["idx"].append([i["idx"].numpy() for i in m.last["infos"]])
        out.setdefault("margin", []).append([_rel_margin(i["dist"]) for i in m.last["infos"]])
    w, vqs = m.state_numpy()
    return cfg, params, vq, out, w, vqs


def main():
    cfg, params, vq, out, w, vqs = run(MICRO, 2, 2, 100)
    arrs = {}
    for s, x in enumerate(out["x"]):
        arrs[f"x{s}"] = x
        for l, idx in enumerate(out["idx"][s]):
            arrs[f"idx{s}_l{l}"] = idx
            arrs[f"margin{s}_l{l}"] = out["margin"][s][l]
        for n, g in out["grads"][s].items():
            arrs[f"grad{s}/{n}"] = g
    for n, v in params.items():
        arrs[f"init/{n}"] = v
    for n, v in w.items():
        arrs[f"final/{n}"] = v
    for l, st in enumerate(vq):
        arrs[f"vq_init{l}/embeddings"] = st["embeddings"]
    for l, st in enumerate(vqs):
        for k in ("embeddings", "m_t", "N_t"):
            arrs[f"vq_final{l}/{k}"] = st[k]
    np.savez_compressed(os.path.join(HERE, "micro.npz"), **arrs)
    json.dump({"config": MICRO, "batch": 2, "steps": 2, "metrics": out["metrics"]},
              open(os.path.join(HERE, "micro.json"), "w"), indent=1)
    # cfg1 (BASELINE config 1): scalars and gradient norms of the first two steps
    cfg, params, vq, out, w, vqs = run(CFG1, 4, 2, 200)
    json.dump({"config": CFG1, "batch": 4, "steps": 2, "x_seeds": [200, 201], "metrics": out["metrics"],
               "grad_norms": [{n: float(np.linalg.norm(g)) for n, g in gs.items()} for gs in out["grads"]],
               "N_t_final": [st["N_t"].tolist() for st in vqs]},
              open(os.path.join(HERE, "cfg1.json"), "w"), indent=1)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
