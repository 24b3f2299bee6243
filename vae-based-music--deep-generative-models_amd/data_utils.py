"""Spectral-loss helpers and the synthetic device feed — the hot-path part of the reference data_utils.py.

data_utils.py:19-22  STFT_ARGS (n_fft, hop_length, window_size) per resolution
data_utils.py:25-30  spectral = |tf.signal.stft(x, frame_length=win, frame_step=hop, fft_length=n_fft)|
data_utils.py:33-40  norm = tf.norm(x, 'fro', axis=[-2, -1])
vqvae.py:309-326     _multispectral_loss = mean_res ||S_x - S_r||_F / ||S_x||_F
The STFT runs on hipFFT (torch.fft) with TF framing: no centering, frame t = x[t*hop : t*hop+win] times
a periodic Hann window, rfft zero-padded at the end to n_fft. The target spectrogram is computed once
per step and shared by all levels (the reference recomputes the same values per level).

File decoding (librosa / GTZAN, data_utils.py:43-206) is out of scope: the north star trains on
synthetic chunks; `synthetic_batch` generates them.
"""
from __future__ import annotations

import math
from typing import List, Tuple

import numpy as np
import torch

STFT_ARGS = [(2048, 1024, 512),  # n_fft
             (240, 120, 50),  # hop_length
             (1200, 600, 240)]  # window_size

_WINDOWS = {}


def _hann(win: int, device) -> torch.Tensor:
    key = (win, str(device))
    if key not in _WINDOWS:
        k = torch.arange(win, dtype=torch.float64)
        _WINDOWS[key] = (0.5 - 0.5 * torch.cos(2 * math.pi * k / win)).to(torch.float32).to(device)
    return _WINDOWS[key]


def spectral(x: torch.Tensor, n_fft: int, hop_length: int, window_length: int) -> torch.Tensor:
    frames = x.unfold(-1, window_length, hop_length)
    return torch.fft.rfft(frames * _hann(window_length, x.device), n=n_fft).abs()


def norm(x: torch.Tensor) -> torch.Tensor:
    return torch.sqrt((x * x).sum(dim=(-2, -1)))


class SpectralTarget:
    """|S_x| and ||S_x||_F for the three resolutions of one batch (B, T, 1) fp32."""

    def __init__(self, x: torch.Tensor):
        t = x.reshape(x.shape[0], -1).float()
        self.specs: List[Tuple[torch.Tensor, torch.Tensor]] = []
        with torch.no_grad():
            for n_fft, hop, win in zip(*STFT_ARGS):
                s = spectral(t, n_fft, hop, win)
                self.specs.append((s, norm(s)))


def multispectral_loss_and_grad(target: SpectralTarget, recon: torch.Tensor):
    """Returns (mean over batch of the per-item multispectral loss, d loss / d recon (B, T, 1) fp32)."""
    r = recon.detach().reshape(recon.shape[0], -1).float().requires_grad_(True)
    with torch.enable_grad():
        losses = []
        for (s_x, n_x), (n_fft, hop, win) in zip(target.specs, zip(*STFT_ARGS)):
            losses.append(norm(s_x - spectral(r, n_fft, hop, win)) / n_x)
        loss = torch.stack(losses, dim=-1).mean(dim=-1).mean()
        (g,) = torch.autograd.grad(loss, r)
    return loss.detach(), g.reshape(recon.shape)


def synthetic_batch(B: int, T: int, sr: int = 44100, seed: int = 1234) -> np.ndarray:
    """clip(0.5 sin(2 pi f t / sr + phi) + 0.05 N(0,1), -1, 1), f ~ U[55, 2000] Hz,
    phi ~ U[0, 2 pi). Shape (B, T, 1) fp32, never silent (the spectral loss has no epsilon)."""
    rng = np.random.default_rng(seed)
    f = rng.uniform(55.0, 2000.0, size=(B, 1))
    ph = rng.uniform(0.0, 2 * np.pi, size=(B, 1))
    t = np.arange(T)[None, :]
    x = 0.5 * np.sin(2 * np.pi * f * t / sr + ph) + 0.05 * rng.standard_normal((B, T))
    return np.clip(x, -1.0, 1.0).astype(np.float32)[:, :, None]
