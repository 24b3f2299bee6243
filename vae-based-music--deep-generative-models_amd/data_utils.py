"""Spectral-loss helpers and the synthetic device feed — the hot-path part of the reference data_utils.py.

data_utils.py:19-22  STFT_ARGS (n_fft, hop_length, window_size) per resolution
data_utils.py:25-30  spectral = |tf.signal.stft(x, frame_length=win, frame_step=hop, fft_length=n_fft)|
data_utils.py:33-40  norm = tf.norm(x, 'fro', axis=[-2, -1])
vqvae.py:309-326     _multispectral_loss = mean_res ||S_x - S_r||_F / ||S_x||_F
The STFT, the loss and its gradient run in libvqa's spectral kernels (csrc/vqa_spectral.hip: in-LDS radix-4
FFTs with TF framing — no centering, frame t = x[t*hop : t*hop+win] times a periodic Hann window, rfft
zero-padded at the end to n_fft).

File decoding (librosa / GTZAN, data_utils.py:43-206) is out of scope: the north star trains on
synthetic chunks. `synthetic_batch_device` generates them in HBM with a HIP kernel (the
device feed); `synthetic_batch` is the numpy restatement the tests and the oracle use.
"""
from __future__ import annotations

import numpy as np
import torch

import vqa_lib as V

STFT_ARGS = [(2048, 1024, 512),  # n_fft
             (240, 120, 50),  # hop_length
             (1200, 600, 240)]  # window_size


def spectral(x: torch.Tensor, n_fft: int, hop_length: int, window_length: int) -> torch.Tensor:
    """data_utils.py:25-30 |tf.signal.stft(x, window_length, hop_length, n_fft)| on the HIP FFT kernel:
    x (..., T) fp32 device tensor -> (..., F, n_fft//2 + 1) fp32."""
    lead, T = tuple(x.shape[:-1]), x.shape[-1]
    xf = x.detach().reshape(-1, T).float().contiguous()
    if window_length > T:
        raise ValueError(f"spectral: signal of {T} samples is shorter than the {window_length}-sample window")
    F = 1 + (T - window_length) // hop_length
    mag = torch.empty(xf.shape[0], F, n_fft // 2 + 1, dtype=torch.float32, device=x.device)
    V.stft_magnitude(xf, mag, n_fft, hop_length, window_length)
    return mag.reshape(*lead, F, n_fft // 2 + 1)


def norm(x: torch.Tensor) -> torch.Tensor:
    """data_utils.py:33-40 tf.norm(x, 'fro', axis=[-2, -1])."""
    return torch.sqrt((x * x).sum(dim=(-2, -1)))


class SpectralTarget:
    """The target waveform of one batch, (B, T) fp32 on the device, and its spectrograms |S_x| for every
    resolution (computed once by vqa_spectral_target and shared by the loss of every level)."""

    def __init__(self, x: torch.Tensor):
        self.x = x.reshape(x.shape[0], -1).float().contiguous()
        self.B, self.T = self.x.shape
        self.mags = V.spectral_target(self.x, *STFT_ARGS)
        self._ws = {}
        # the spectrograms are complete when this event (on the producing stream) has fired: a loss on another
        # stream waits for it (the levels' streams only need the target at their losses, not at their start)
        self.ready = None
        if self.x.is_cuda:
            self._stream = torch.cuda.current_stream(self.x.device)
            self.ready = torch.cuda.Event()
            self.ready.record(self._stream)

    def wait(self):
        """Order the current stream after the spectrograms (no-op on the producing stream)."""
        if self.ready is not None:
            cur = torch.cuda.current_stream(self.x.device)
            if cur != self._stream:
                cur.wait_event(self.ready)

    def workspace(self, grad: bool) -> torch.Tensor:
        """Loss scratch, one per stream (levels on concurrent streams never share it)."""
        key = (grad, torch.cuda.current_stream(self.x.device).cuda_stream if self.x.is_cuda else 0)
        if key not in self._ws:
            n = V.spectral_loss_target_workspace(self.B, self.T, *STFT_ARGS, with_grad=grad)
            self._ws[key] = V.workspace(n, self.x.device)
        return self._ws[key]


def multispectral_loss_and_grad(target: SpectralTarget, recon: torch.Tensor, loss_out=None, need_grad=True):
    """vqvae.py:309-326 _multispectral_loss (mean over the batch of the per-item mean over resolutions) and
    its gradient d loss / d recon, (B, T, 1) fp32 — one vqa_spectral_loss_target call against the shared
    target spectrograms. Returns (loss (1,), grad)."""
    r = recon.reshape(recon.shape[0], -1)
    if r.dtype != torch.float32:
        raise ValueError("the multispectral loss takes the fp32 reconstruction")
    if r.shape != target.x.shape:
        raise ValueError(f"reconstruction {tuple(r.shape)} vs target {tuple(target.x.shape)}")
    loss = loss_out if loss_out is not None else torch.empty(1, dtype=torch.float32, device=r.device)
    dr = torch.empty_like(r) if need_grad else None
    target.wait()
    V.spectral_loss_target(target.mags, r.contiguous(), loss, dr, None, *STFT_ARGS, ws=target.workspace(need_grad))
    return loss, (dr.reshape(recon.shape) if need_grad else None)


def splitsongs(X, y, window=0.05, overlap=0.5):
    """data_utils.py:65-91: a song cut into overlapping chunks of int(T * window) samples, hopping by
    int(chunk * (1 - overlap)); a chunk that would run past the end is dropped. X is (T,) or (C, T); returns
    ((n, chunk) or (n, C, chunk), (n,) copies of the label) — channels first, as the reference's callers then
    transpose to (B, T, C). Host numpy, like the reference (the training feed itself is generated on the
    device: synthetic_batch_device)."""
    X = np.asarray(X)
    T = X.shape[-1]
    chunk = int(T * window)
    hop = int(chunk * (1.0 - overlap))
    pieces = [X[..., s:s + chunk] for s in range(0, T - chunk + hop, hop)]
    pieces = [p for p in pieces if p.shape[-1] == chunk]
    return np.array(pieces), np.array([y] * len(pieces))


def synthetic_batch(B: int, T: int, sr: int = 44100, seed: int = 1234) -> np.ndarray:
    """clip(0.5 sin(2 pi f t / sr + phi) + 0.05 N(0,1), -1, 1), f ~ U[55, 2000] Hz,
    phi ~ U[0, 2 pi). Shape (B, T, 1) fp32, never silent (the spectral loss has no epsilon)."""
    rng = np.random.default_rng(seed)
    f = rng.uniform(55.0, 2000.0, size=(B, 1))
    ph = rng.uniform(0.0, 2 * np.pi, size=(B, 1))
    t = np.arange(T)[None, :]
    x = 0.5 * np.sin(2 * np.pi * f * t / sr + ph) + 0.05 * rng.standard_normal((B, T))
    return np.clip(x, -1.0, 1.0).astype(np.float32)[:, :, None]


def synthetic_batch_device(B: int, T: int, seed: int = 1234, rank: int = 0, sr: float = 44100.0,
                           device="cuda", out: torch.Tensor = None) -> torch.Tensor:
    """The same distribution generated on the GPU (vqa_synthetic_batch: counter-based draws keyed by seed,
    rank, item and sample), (B, T, 1) fp32 resident in HBM — the device feed of the train step; no host
    staging. Deterministic per (seed, rank); ranks draw disjoint streams."""
    x = out if out is not None else torch.empty(B, T, 1, dtype=torch.float32, device=device)
    V.synthetic_batch(x, seed, rank, sr)
    return x
