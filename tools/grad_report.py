"""Per-tensor gradient error of one fp32 GPU train step vs the fp64 oracle (debugging aid).
usage: python tools/grad_report.py [cfg1|cfg2_short|tiny]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np, torch
from oracle import vqvae_ref as R
from test_gpu_train import CONFIGS, _model

name = sys.argv[1] if len(sys.argv) > 1 else "cfg1"
cfg, B = CONFIGS[name]["cfg"], CONFIGS[name]["B"]
params, vq = R.init_params(cfg, 1), R.init_vq_state(cfg, 2)
x = R.synthetic_batch(B, cfg.input_len, seed=11)
ref = R.RefVQVAE(cfg, params, vq, dtype=torch.float64)
m = _model(cfg, B, "fp32", params, vq)
ref.train_step(x)
m.train_step(x)
g = m.store.grads()
rows = []
for n, r in ref.last["grads"].items():
    r = r.numpy()
    rows.append((float(np.max(np.abs(g[n] - r)) / max(np.max(np.abs(r)), 1e-30)), n))
rows.sort()
print("median", np.median([e for e, _ in rows]))
for e, n in rows[::max(1, len(rows) // 25)] + rows[-5:]:
    print(f"{e:.2e} {n}")
