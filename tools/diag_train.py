"""Diagnostic: where does the fp32 train-step gradient diverge from the fp64 oracle?"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]
import numpy as np, torch
from oracle import vqvae_ref as R
from vqvae import VQVAE

cfg = R.RefConfig(input_len=4096, levels=1, latent_dim=64, down_depth=[3], strides=[2], num_embeddings=256,
                  residual_width=32, residual_depth=4, dilation_factor=3)
B = 4
params, vq = R.init_params(cfg, 1), R.init_vq_state(cfg, 2)
x = R.synthetic_batch(B, cfg.input_len, seed=11)
for dt in ("fp32", "bf16"):
    ref = R.RefVQVAE(cfg, params, vq, dtype=torch.float64)
    m = VQVAE((cfg.input_len, 1), 1, 64, [3], [2], num_embeddings=256, residual_width=32, residual_depth=4,
              dilation_factor=3, dtype=dt, device="cuda:0")
    m.set_weights(params); m.set_vq_state(vq); m.compile()
    # encoder output & indices
    xt = torch.from_numpy(x).cuda()
    z = m.encoders[0].forward(xt)
    zr = ref.encoder(torch.from_numpy(x).double(), 0).detach()
    print(dt, "z rel err", float((z.double().cpu() - zr).abs().max() / zr.abs().max()))
    idx = m.vqs[0].get_code_indices(z.reshape(-1, 64)).cpu()
    E = torch.from_numpy(vq[0]["embeddings"]).double()
    d = (zr.reshape(-1, 64) ** 2).sum(1, keepdim=True) + (E ** 2).sum(0) - 2 * zr.reshape(-1, 64) @ E
    ridx = d.argmin(1)
    top2 = torch.topk(d, 2, dim=1, largest=False).values
    mis = (idx != ridx)
    print(dt, "index mismatches", int(mis.sum()), "of", len(idx), "margins of mismatches",
          (top2[mis, 1] - top2[mis, 0]).numpy()[:10])
    m.train_step(x)
    ref.train_step(x)
    g = m.store.grads()
    errs = sorted(((float(np.max(np.abs(g[n] - r.numpy())) / max(np.max(np.abs(r.numpy())), 1e-12)), n)
                   for n, r in ref.last["grads"].items()), reverse=True)
    for e, n in errs[:8]:
        print(f"  {dt} {n:40s} {e:.3e}")
    print(dt, "median grad rel err", np.median([e for e, _ in errs]))
