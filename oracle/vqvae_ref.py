"""CPU restatement of the reference's VQ-VAE training step (torch CPU, fp64 or fp32). TEST INFRASTRUCTURE ONLY.

It keeps the reference's op sequence and costs on purpose — dense one-hot GEMMs, a materialised N x K
distance matrix, TF-style STFT framing — because it doubles as bench.py's CPU baseline ("port").
Gradients come from torch autograd (independent of the product's hand-written backward).

Follows, line by line:
  resnet.py:7-59        ResnetConv1DBlock / DilatedResnet1D             -> res_block, dilated_resnet
  encdec.py:17-151      EncoderConvBlock / DecoderConvBlock / Encoder / Decoder -> encoder, decoder
  VectorQuantizer.py:8-199  EMA vector quantizer                         -> vq_forward
  vqvae.py:15-21,30-146,148-260,309-326  VQVAE (train_step, test_step, call, encode, decode, losses)
  data_utils.py:19-40   STFT_ARGS / spectral / norm                       -> spectral, norm
  keras 2.7 Adam (vqvae.py:144,362) via TF ApplyAdam                       -> keras_adam
TF semantics restated here are pinned by tests/test_oracle_kat.py.
Parity with TensorFlow itself is UNPINNED (TF is not importable here; see oracle/__init__.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from . import reset_perm

# data_utils.py:19-22 — (n_fft, hop_length, window_size) per resolution
STFT_ARGS = [(2048, 240, 1200), (1024, 120, 600), (512, 50, 240)]


# ---------------------------------------------------------------------------------------------------
# TF semantics

def same_pad(T: int, K: int, stride: int, dilation: int = 1) -> Tuple[int, int, int]:
    """TF 'SAME': out = ceil(T/s); pad = max((out-1)*s + (K-1)*d + 1 - T, 0); left = pad // 2."""
    out = -(-T // stride)
    pad = max((out - 1) * stride + (K - 1) * dilation + 1 - T, 0)
    return out, pad // 2, pad - pad // 2


def conv1d(x, W, b, stride=1, dilation=1):
    """keras Conv1D(padding='same'): x (B,T,Cin), W (K,Cin,Cout) -> (B,ceil(T/s),Cout)."""
    B, T, C = x.shape
    K = W.shape[0]
    _, pl, pr = same_pad(T, K, stride, dilation)
    xt = F.pad(x.transpose(1, 2), (pl, pr))
    y = F.conv1d(xt, W.permute(2, 1, 0), b, stride=stride, dilation=dilation)
    return y.transpose(1, 2)


def conv1d_transpose(x, W, b, stride):
    """keras Conv1DTranspose(padding='same'): the adjoint of the SAME conv on the stride*T signal.
    x (B,T,Cin), W (K,Cout,Cin) -> (B, stride*T, Cout)."""
    B, T, C = x.shape
    K = W.shape[0]
    Tout = stride * T
    _, pl, _ = same_pad(Tout, K, stride, 1)
    full = F.conv_transpose1d(x.transpose(1, 2), W.permute(2, 1, 0), None, stride=stride)
    y = full[:, :, pl:pl + Tout] + b[None, :, None]
    return y.transpose(1, 2)


def hann_periodic(n: int, dtype=torch.float64):
    """tf.signal.hann_window(n, periodic=True) = 0.5 - 0.5*cos(2*pi*k/n)."""
    k = torch.arange(n, dtype=torch.float64)
    return (0.5 - 0.5 * torch.cos(2 * math.pi * k / n)).to(dtype)


def spectral(x, n_fft, hop, win):
    """data_utils.spectral: |tf.signal.stft(x, win, hop, n_fft)| — no centering, frame t starts at
    t*hop, periodic Hann of length win, rfft zero-padded at the end to n_fft. x (..., T)."""
    frames = x.unfold(-1, win, hop)
    return torch.fft.rfft(frames * hann_periodic(win, x.dtype), n=n_fft).abs()


def norm(x):
    """data_utils.norm: tf.norm(x, ord='fro', axis=[-2, -1])."""
    return torch.sqrt((x * x).sum(dim=(-2, -1)))


def multispectral_loss(target, recon):
    """vqvae.py:309-326 on (B,T,1) tensors -> (B,) per-item mean over resolutions."""
    t = target.squeeze(-1)
    r = recon.squeeze(-1)
    losses = []
    for n_fft, hop, win in STFT_ARGS:
        st = spectral(t, n_fft, hop, win)
        sr = spectral(r, n_fft, hop, win)
        losses.append(norm(st - sr) / norm(st))
    return torch.stack(losses, dim=-1).mean(dim=-1)


def keras_adam(w, g, m, v, t, lr=1e-3, b1=0.9, b2=0.999, eps=1e-7, alpha=None):
    """TF ApplyAdam as used by keras 2.7 Adam; t is the 1-based step. Returns (w, m, v). `alpha` overrides the
    step size lr*sqrt(1-b2^t)/(1-b1^t) (e.g. with TF's float32 evaluation of the powers, adam_alpha_f32)."""
    if alpha is None:
        alpha = lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    m = m + (g - m) * (1 - b1)
    v = v + (g * g - v) * (1 - b2)
    w = w - (m * alpha) / (torch.sqrt(v) + eps)
    return w, m, v


def adam_alpha_f32(lr, t, b1=0.9, b2=0.999):
    """Keras Adam's step size as TF computes it: every hyper-parameter and beta^t in float32
    (OptimizerV2 Adam._prepare_local: beta_2_power = pow(beta_2_t, local_step) in the variable dtype), so
    1 - beta_2^t carries float32 cancellation at small t (~3e-5 relative at t = 2)."""
    f = np.float32
    b1p, b2p = f(f(b1) ** f(t)), f(f(b2) ** f(t))
    return float(f(f(lr) * f(np.sqrt(f(f(1) - b2p)))) / f(f(1) - b1p))


# ---------------------------------------------------------------------------------------------------
# model structure

@dataclass
class RefConfig:
    input_len: int
    levels: int
    latent_dim: int
    down_depth: Sequence[int]
    strides: Sequence[int]
    num_embeddings: int = 128
    residual_width: int = 64
    residual_depth: int = 4
    dilation_factor: int = 1
    beta: float = 0.25
    decay: float = 0.99
    threshold: float = 1.0
    reset_seed: int = 3


def param_specs(cfg: RefConfig) -> List[Tuple[str, Tuple[int, ...]]]:
    """Canonical (name, shape) list in build order: vqvae.py:47-74 -> encdec.py -> resnet.py."""
    D, W, R = cfg.latent_dim, cfg.residual_width, cfg.residual_depth
    specs = []

    def conv(name, K, cin, cout):
        specs.append((f"{name}/kernel", (K, cin, cout)))
        specs.append((f"{name}/bias", (cout,)))

    def convT(name, K, cin, cout):
        specs.append((f"{name}/kernel", (K, cout, cin)))
        specs.append((f"{name}/bias", (cout,)))

    def res(prefix):
        for j in range(R):
            conv(f"{prefix}/rb{j}/conv_a", 3, W, W)
            conv(f"{prefix}/rb{j}/conv_b", 3, W, W)

    for l in range(cfg.levels):
        for b in range(l + 1):
            s = cfg.strides[b]
            for i in range(cfg.down_depth[b]):
                cin = (1 if b == 0 else D) if i == 0 else W
                conv(f"enc{l}/blk{b}/down{i}", 2 * s, cin, W)
                res(f"enc{l}/blk{b}/res{i}")
            conv(f"enc{l}/blk{b}/proj", 3, W, D)
        for b in reversed(range(l + 1)):
            s = cfg.strides[b]
            conv(f"dec{l}/blk{b}/pre", 3, D, W)
            for i in range(cfg.down_depth[b]):
                res(f"dec{l}/blk{b}/res{i}")
                cout = D if i == cfg.down_depth[b] - 1 else W
                convT(f"dec{l}/blk{b}/up{i}", 2 * s, W, cout)
        conv(f"dec{l}/out", 3, D, 1)
    return specs


def init_params(cfg: RefConfig, seed: int = 1) -> Dict[str, np.ndarray]:
    """keras defaults: glorot_uniform kernels (limit sqrt(6/(K*s[1] + K*s[2]))), zero biases."""
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in param_specs(cfg):
        if name.endswith("/kernel"):
            K = shape[0]
            lim = math.sqrt(6.0 / (K * shape[1] + K * shape[2]))
            out[name] = rng.uniform(-lim, lim, size=shape).astype(np.float32)
        else:
            out[name] = np.zeros(shape, np.float32)
    return out


def init_vq_state(cfg: RefConfig, seed: int = 2) -> List[Dict[str, np.ndarray]]:
    """VectorQuantizer.py:38-60: E ~ U(-0.05, 0.05) (D, K); m_t = E; N_t = ones(K)."""
    rng = np.random.default_rng(seed)
    st = []
    for _ in range(cfg.levels):
        E = rng.uniform(-0.05, 0.05, size=(cfg.latent_dim, cfg.num_embeddings)).astype(np.float32)
        st.append({"embeddings": E, "m_t": E.copy(), "N_t": np.ones(cfg.num_embeddings, np.float32),
                   "calls": 0})
    return st


# ---------------------------------------------------------------------------------------------------

class RefVQVAE:
    """The reference VQVAE (vqvae.py:24-326) restated on torch CPU."""

    def __init__(self, cfg: RefConfig, params: Dict[str, np.ndarray], vq_state, dtype=torch.float64):
        self.cfg = cfg
        self.dtype = dtype
        self.p = {k: torch.tensor(np.asarray(v), dtype=dtype, requires_grad=True) for k, v in params.items()}
        self.names = [n for n, _ in param_specs(cfg)]
        self.vq = [{"embeddings": torch.tensor(np.asarray(s["embeddings"]), dtype=dtype),
                    "m_t": torch.tensor(np.asarray(s["m_t"]), dtype=dtype),
                    "N_t": torch.tensor(np.asarray(s["N_t"]), dtype=dtype),
                    "calls": int(s.get("calls", 0))} for s in vq_state]
        self.adam_m = {k: torch.zeros_like(v) for k, v in self.p.items()}
        self.adam_v = {k: torch.zeros_like(v) for k, v in self.p.items()}
        self.iterations = 0
        self.last = {}
        if dtype == torch.float32:
            self.gamma = float(np.float32(cfg.decay))
            self.omg = float(np.float32(1.0 - cfg.decay))
        else:
            self.gamma, self.omg = cfg.decay, 1.0 - cfg.decay

    # resnet.py:7-29
    def res_block(self, x, pfx, dilation):
        h = conv1d(F.relu(x), self.p[f"{pfx}/conv_a/kernel"], self.p[f"{pfx}/conv_a/bias"], 1, dilation)
        y = conv1d(F.relu(h), self.p[f"{pfx}/conv_b/kernel"], self.p[f"{pfx}/conv_b/bias"], 1, 1)
        return x + y

    # resnet.py:40-59 (dilation_cycle=None); decoder stacks are reversed (:54-55)
    def dilated_resnet(self, x, pfx, reverse):
        R, f = self.cfg.residual_depth, self.cfg.dilation_factor
        for j in range(R):
            d = f ** (R - 1 - j) if reverse else f ** j
            x = self.res_block(x, f"{pfx}/rb{j}", d)
        return x

    # encdec.py:74-108 with EncoderConvBlock :17-41
    def encoder(self, x, l):
        for b in range(l + 1):
            s = self.cfg.strides[b]
            for i in range(self.cfg.down_depth[b]):
                x = conv1d(x, self.p[f"enc{l}/blk{b}/down{i}/kernel"], self.p[f"enc{l}/blk{b}/down{i}/bias"], s, 1)
                x = self.dilated_resnet(x, f"enc{l}/blk{b}/res{i}", False)
            x = conv1d(x, self.p[f"enc{l}/blk{b}/proj/kernel"], self.p[f"enc{l}/blk{b}/proj/bias"], 1, 1)
        return x

    # encdec.py:114-151 with DecoderConvBlock :44-71
    def decoder(self, x, l):
        for b in reversed(range(l + 1)):
            s = self.cfg.strides[b]
            x = conv1d(x, self.p[f"dec{l}/blk{b}/pre/kernel"], self.p[f"dec{l}/blk{b}/pre/bias"], 1, 1)
            for i in range(self.cfg.down_depth[b]):
                x = self.dilated_resnet(x, f"dec{l}/blk{b}/res{i}", True)
                x = conv1d_transpose(x, self.p[f"dec{l}/blk{b}/up{i}/kernel"], self.p[f"dec{l}/blk{b}/up{i}/bias"], s)
        return conv1d(x, self.p[f"dec{l}/out/kernel"], self.p[f"dec{l}/out/bias"], 1, 1)

    # VectorQuantizer.py:75-186
    def vq_forward(self, z, l, training):
        st = self.vq[l]
        E = st["embeddings"]
        D, K = E.shape
        flat = z.reshape(-1, D)
        with torch.no_grad():
            fd = flat.detach()
            sim = fd @ E
            dist = (fd ** 2).sum(dim=1, keepdim=True) + (E ** 2).sum(dim=0) - 2 * sim
            idx = torch.argmin(dist, dim=1)
        enc = F.one_hot(idx, K).to(self.dtype)
        q = enc @ E.T
        commit = self.cfg.beta * ((q.detach() - flat) ** 2).mean()
        q_st = flat + (q - flat).detach()
        info = {"idx": idx, "dist": dist, "commit": commit}
        if training:
            with torch.no_grad():
                m_sum = fd.T @ enc
                n_sum = enc.sum(dim=0)
                st["m_t"] = self.gamma * st["m_t"] + self.omg * m_sum
                st["N_t"] = self.gamma * st["N_t"] + self.omg * n_sum
                usage = (st["N_t"] >= self.cfg.threshold).to(self.dtype).reshape(1, K)
                rows = reset_perm.reset_rows(self.cfg.reset_seed, st["calls"], l, fd.shape[0], K)
                random_codes = fd[torch.from_numpy(rows)].T
                st["embeddings"] = usage * (st["m_t"] / st["N_t"].clamp(1e-8, 1e8).reshape(1, K)) + \
                    (1.0 - usage) * random_codes
                st["calls"] += 1
                p = n_sum / n_sum.sum()
                info.update({"m_sum": m_sum, "n_sum": n_sum, "reset_rows": rows,
                             "batch_usage": float((n_sum >= self.cfg.threshold).sum()),
                             "usage": float((st["N_t"] >= self.cfg.threshold).sum()),
                             "entropy": float(-(p * torch.log(p + 1e-8)).sum())})
        return q_st.reshape(z.shape), idx, info

    def level_forward(self, x, l, training):
        z = self.encoder(x, l)
        q_st, idx, info = self.vq_forward(z, l, training)
        recon = self.decoder(q_st, l)
        recon_loss = ((x - recon) ** 2).mean()
        spec_loss = multispectral_loss(x, recon).mean()
        commit = info["commit"]
        info.update({"z": z, "q_st": q_st, "recon": recon, "recon_loss": recon_loss, "spectral_loss": spec_loss,
                     "level_loss": recon_loss + commit + spec_loss})
        return info

    def forward_losses(self, x, training):
        x = torch.as_tensor(np.asarray(x), dtype=self.dtype)
        infos = [self.level_forward(x, l, training) for l in range(self.cfg.levels)]
        total = torch.zeros((), dtype=self.dtype)
        for inf in infos:
            total = total + inf["level_loss"]
        return total, infos

    def train_step(self, x, lr=1e-3):
        """vqvae.py:111-146 (+ keras Adam). Returns per-step scalars; keeps infos/grads in self.last."""
        total, infos = self.forward_losses(x, training=True)
        params = [self.p[n] for n in self.names]
        grads = torch.autograd.grad(total, params)
        self.iterations += 1
        with torch.no_grad():
            for n, g in zip(self.names, grads):
                w, m, v = keras_adam(self.p[n].detach(), g, self.adam_m[n], self.adam_v[n], self.iterations, lr=lr)
                self.p[n] = w.clone().requires_grad_(True)
                self.adam_m[n], self.adam_v[n] = m, v
        self.last = {"total": total.detach(), "infos": infos, "grads": dict(zip(self.names, grads))}
        return self._scalars(total, infos)

    def test_step(self, x):
        """vqvae.py:148-172 — the VQ runs with its default training=True, so the EMA updates."""
        with torch.no_grad():
            total, infos = self.forward_losses(x, training=True)
        self.last = {"total": total, "infos": infos}
        return self._scalars(total, infos)

    def call(self, x, training=False):
        """vqvae.py:178-206."""
        with torch.no_grad():
            total, infos = self.forward_losses(x, training=training)
        return [i["recon"] for i in infos], {"level_losses": [i["level_loss"] for i in infos],
                                              "recon_losses": [i["recon_loss"] for i in infos],
                                              "commit_losses": [i["commit"] for i in infos],
                                              "spec_losses": [i["spectral_loss"] for i in infos]}

    def encode(self, x, start_level=0, end_level=None):
        """vqvae.py:208-236."""
        end_level = self.cfg.levels if end_level is None else end_level
        x = torch.as_tensor(np.asarray(x), dtype=self.dtype)
        out = []
        with torch.no_grad():
            for l in range(start_level, end_level):
                z = self.encoder(x, l)
                _, idx, _ = self.vq_forward(z, l, training=False)
                out.append(idx.reshape(z.shape[:-1]))
        return out

    def decode(self, zq, level=0):
        """vqvae.py:238-260."""
        st = self.vq[level]
        with torch.no_grad():
            q = F.one_hot(torch.as_tensor(zq), st["embeddings"].shape[1]).to(self.dtype) @ st["embeddings"].T
            return self.decoder(q, level)

    @staticmethod
    def _scalars(total, infos):
        f = lambda v: float(v.detach()) if isinstance(v, torch.Tensor) else float(v)  # noqa: E731
        out = {"loss": f(total)}
        out["recon_loss"] = sum(f(i["recon_loss"]) for i in infos)
        out["vqvae_loss"] = sum(f(i["commit"]) for i in infos)
        out["spectral_loss"] = sum(f(i["spectral_loss"]) for i in infos)
        for l, i in enumerate(infos):
            out[f"[{l}]level_loss"] = f(i["level_loss"])
            out[f"[{l}]recon_loss"] = f(i["recon_loss"])
            out[f"[{l}]vq_loss"] = f(i["commit"])
            out[f"[{l}]spectral_loss"] = f(i["spectral_loss"])
            for k in ("batch_usage", "usage", "entropy"):
                if k in i:
                    key = {"batch_usage": "batch_codebook_usage", "usage": "codebook_usage",
                           "entropy": "codebook_entropy"}[k]
                    out[f"[{l}]{key}"] = i[k]
        return out

    def state_numpy(self):
        return ({k: v.detach().numpy().copy() for k, v in self.p.items()},
                [{"embeddings": s["embeddings"].numpy().copy(), "m_t": s["m_t"].numpy().copy(),
                  "N_t": s["N_t"].numpy().copy(), "calls": s["calls"]} for s in self.vq])


def synthetic_batch(B: int, T: int, sr: int = 44100, seed: int = 1234) -> np.ndarray:
    """SURVEY.md §8d synthetic feed: clip(0.5 sin(2 pi f t/sr + phi) + 0.05 N(0,1), -1, 1), (B,T,1) fp32."""
    rng = np.random.default_rng(seed)
    f = rng.uniform(55.0, 2000.0, size=(B, 1))
    ph = rng.uniform(0.0, 2 * np.pi, size=(B, 1))
    t = np.arange(T)[None, :]
    x = 0.5 * np.sin(2 * np.pi * f * t / sr + ph) + 0.05 * rng.standard_normal((B, T))
    return np.clip(x, -1.0, 1.0).astype(np.float32)[:, :, None]
