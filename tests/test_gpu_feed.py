"""On-device synthetic feed (vqa_synthetic_batch; SURVEY.md §8d, replacing the host chunk feed of
data_utils.py:65-206) against the numpy generator `synthetic_batch` it stands in for: same value distribution
(two-sample KS distance), one sinusoid per item with f in [55, 2000) Hz carrying ~98 % of the power, noise of
variance 0.05^2 around it, clipping to [-1, 1]; deterministic per (seed, rank), disjoint across ranks and seeds.
The draws are a counter-based hash (not numpy's PCG64 stream), so the comparison is distributional."""
import numpy as np
import pytest
import torch

from data_utils import synthetic_batch, synthetic_batch_device

pytestmark = pytest.mark.gpu


def _ks(a, b):
    a, b = np.sort(a), np.sort(b)
    grid = np.concatenate([a, b])
    return float(np.max(np.abs(np.searchsorted(a, grid, "right") / len(a) - np.searchsorted(b, grid, "right") / len(b))))


def test_feed_distribution_matches_numpy_generator(cuda):
    B, T, sr = 64, 65536, 44100
    x = synthetic_batch_device(B, T, seed=1234, rank=0, device=cuda).cpu().numpy()[:, :, 0]
    ref = synthetic_batch(B, T, seed=1234)[:, :, 0]
    assert x.shape == (B, T) and x.dtype == np.float32
    assert np.abs(x).max() <= 1.0 and np.isfinite(x).all()
    sub = np.random.default_rng(0).choice(B * T, 200000, replace=False)
    assert _ks(x.reshape(-1)[sub], ref.reshape(-1)[sub]) < 0.02
    assert abs(x.mean()) < 0.01 and abs(x.std() - ref.std()) < 0.01
    w = np.hanning(T + 1)[:T]  # windowed periodogram: the sinusoid's leakage stays within a few bins
    spec = np.abs(np.fft.rfft(x.astype(np.float64) * w, axis=1)) ** 2
    freqs = np.fft.rfftfreq(T, 1 / sr)
    peak = spec.argmax(1)
    assert ((freqs[peak] >= 54) & (freqs[peak] <= 2001)).all()
    band = np.zeros_like(spec, dtype=bool)
    for b in range(B):
        band[b, max(peak[b] - 8, 0):peak[b] + 9] = True
    frac = (spec * band).sum(1) / spec.sum(1)
    assert (frac > 0.95).all(), frac.min()  # 0.125 / (0.125 + 0.0025) = 0.98 of the power is the sinusoid
    noise_var = (spec * ~band).sum(1) / (~band).sum(1) / (w ** 2).sum()  # white noise: E|X_k|^2 = var * sum w^2
    assert np.all((noise_var > 0.05 ** 2 * 0.8) & (noise_var < 0.05 ** 2 * 1.2)), (noise_var.min(), noise_var.max())
    # item frequencies spread over the band (uniform: mean ~1027 Hz)
    assert 700 < freqs[peak].mean() < 1350


def test_feed_deterministic_per_seed_and_rank(cuda):
    a = synthetic_batch_device(4, 10000, seed=7, rank=0, device=cuda)
    b = synthetic_batch_device(4, 10000, seed=7, rank=0, device=cuda)
    c = synthetic_batch_device(4, 10000, seed=7, rank=1, device=cuda)
    d = synthetic_batch_device(4, 10000, seed=8, rank=0, device=cuda)
    assert torch.equal(a, b)
    assert not torch.equal(a, c) and not torch.equal(a, d)
    # a prefix of a longer chunk is the shorter chunk (draws keyed by sample index)
    e = synthetic_batch_device(4, 20000, seed=7, rank=0, device=cuda)
    assert torch.equal(e[:, :10000], a)
