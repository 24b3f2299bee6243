"""Spectral-loss kernel parity (vqa_spectral.hip) vs the CPU oracle in fp64.

Follows data_utils.py:25-40 (spectral / norm) and vqvae.py:309-326 (_multispectral_loss); the oracle's
gradient is torch autograd through rfft/abs (abs'(0) = 0, as TF). Tolerances (fp32 FFT vs fp64):
magnitudes 2e-6 of the spectrum's max, loss 1e-5 relative, gradient 1e-4 of its max-abs.
"""
import numpy as np
import pytest
import torch

import vqa_lib as V
from data_utils import STFT_ARGS, SpectralTarget, multispectral_loss_and_grad, spectral
from oracle import vqvae_ref as R

pytestmark = pytest.mark.gpu

RES = list(zip(*STFT_ARGS))  # (n_fft, hop, win) per resolution


def _signals(B, T, seed, recon_scale=0.3):
    x = torch.from_numpy(R.synthetic_batch(B, T, seed=seed))
    g = torch.Generator().manual_seed(seed + 1)
    r = recon_scale * torch.randn(B, T, 1, generator=g) + 0.5 * x
    return x, r


def _oracle(x, r):
    rd = r.double().clone().requires_grad_(True)
    per_item = R.multispectral_loss(x.double(), rd)
    loss = per_item.mean()
    (g,) = torch.autograd.grad(loss, rd)
    return float(loss.detach()), per_item.detach(), g


@pytest.mark.parametrize("n_fft,hop,win", RES + [(256, 64, 256), (512, 100, 300), (1024, 1, 7)])
def test_stft_magnitude(cuda, n_fft, hop, win):
    x, _ = _signals(3, 4096 + 37, seed=n_fft + win)
    got = spectral(x.squeeze(-1).to(cuda), n_fft, hop, win).cpu().double()
    ref = R.spectral(x.squeeze(-1).double(), n_fft, hop, win)
    assert got.shape == ref.shape
    err = (got - ref).abs().max() / ref.abs().max()
    assert err < 2e-6, err


@pytest.mark.parametrize("B,T", [(2, 8192), (3, 4096 + 113), (1, 1200), (4, 2048)])
def test_loss_and_grad(cuda, B, T):
    x, r = _signals(B, T, seed=B * 1000 + T)
    loss_ref, item_ref, g_ref = _oracle(x, r)
    tgt = SpectralTarget(x.to(cuda))
    loss, dr = multispectral_loss_and_grad(tgt, r.to(cuda))
    assert abs(float(loss) - loss_ref) / loss_ref < 1e-5
    g = dr.cpu().double()
    assert g.shape == g_ref.shape
    err = (g - g_ref).abs().max() / g_ref.abs().max()
    assert err < 1e-4, err
    # per-item losses through the C-ABI's item_loss output
    item = torch.empty(B, device=cuda)
    out = torch.empty(1, device=cuda)
    V.spectral_loss(tgt.x, r.to(cuda).reshape(B, T).contiguous(), out, None, item, *STFT_ARGS)
    assert torch.allclose(item.cpu().double(), item_ref, rtol=1e-5)
    assert float(out) == float(loss)  # loss-only mode = the same reduction


def test_full_size_deterministic(cuda):
    """cfg2 chunk length: bit-identical repeat, and loss/grad vs the oracle on 2 of the 32 items."""
    B, T = 32, 65536
    x, r = _signals(B, T, seed=7)
    tgt = SpectralTarget(x.to(cuda))
    rd = r.to(cuda)
    l1, g1 = multispectral_loss_and_grad(tgt, rd)
    l2, g2 = multispectral_loss_and_grad(tgt, rd)
    assert torch.equal(l1, l2) and torch.equal(g1, g2)
    # items are independent: the batch-mean gradient of item b is (1/B) x its single-item gradient
    sub = [0, 31]
    loss_ref, item_ref, g_ref = _oracle(x[sub], r[sub])
    item = torch.empty(B, device=cuda)
    V.spectral_loss(tgt.x, rd.reshape(B, T), torch.empty(1, device=cuda), None, item, *STFT_ARGS)
    assert torch.allclose(item.cpu().double()[sub], item_ref, rtol=1e-5)
    g = g1.cpu().double()[sub] * (B / len(sub))
    err = (g - g_ref).abs().max() / g_ref.abs().max()
    assert err < 1e-4, err


def test_zero_bins_gradient(cuda):
    """abs'(0) = 0: a reconstruction that is exactly zero has zero spectral gradient (no NaN)."""
    B, T = 2, 4096
    x, _ = _signals(B, T, seed=3)
    r = torch.zeros(B, T, 1)
    loss, dr = multispectral_loss_and_grad(SpectralTarget(x.to(cuda)), r.to(cuda))
    assert abs(float(loss) - 1.0) < 1e-6  # ||S_x - 0|| / ||S_x||
    assert torch.count_nonzero(dr).item() == 0


def test_bad_shapes(cuda):
    x = torch.zeros(2, 1000, device=cuda)
    with pytest.raises(V.VQAError):
        V.spectral_loss_workspace(2, 1000, *STFT_ARGS)  # 1000 < win 1200
    with pytest.raises(V.VQAError):
        V.stft_magnitude(x, torch.empty(1, device=cuda), 4096, 10, 100)  # n_fft unsupported


@pytest.mark.parametrize("B,T", [(3, 4096 + 113), (2, 65536)])
def test_shared_target(cuda, B, T):
    """One vqa_spectral_target buffer serves several reconstructions (the levels of a train step) and gives
    the same bits as the one-call vqa_spectral_loss; odd frame counts exercise the unpaired last frame."""
    x, r = _signals(B, T, seed=11 + T)
    tgt = SpectralTarget(x.to(cuda))
    for k, scale in enumerate((0.3, 0.05)):
        rr = (scale * torch.randn(B, T, 1, generator=torch.Generator().manual_seed(k)) + 0.5 * x).to(cuda)
        l1, g1 = multispectral_loss_and_grad(tgt, rr)
        l0 = torch.empty(1, device=cuda)
        g0 = torch.empty(B, T, device=cuda)
        V.spectral_loss(tgt.x, rr.reshape(B, T), l0, g0, None, *STFT_ARGS)
        assert torch.equal(l0, l1) and torch.equal(g0, g1.reshape(B, T))
        l2, _ = multispectral_loss_and_grad(tgt, rr, need_grad=False)
        assert torch.equal(l1, l2)
    if T < 10000:
        loss_ref, _, g_ref = _oracle(x, rr.cpu())
        assert abs(float(l1) - loss_ref) / loss_ref < 1e-5
        err = (g1.cpu().double() - g_ref).abs().max() / g_ref.abs().max()
        assert err < 1e-4, err


@pytest.mark.parametrize("args", [
    [(512, 256), (20, 64), (300, 256)],                 # 15 frames over a sample: the general overlap-add
    [(2048, 1024, 512, 256, 512), (240, 120, 50, 64, 100), (1200, 600, 240, 256, 300)],  # 5 resolutions
    [(256,), (1,), (7,)],                                # hop 1
    [tuple(a) for a in STFT_ARGS],                       # the model's: the 8-frame gather
])
def test_gradient_overlap_add_forms(cuda, args):
    """The frame-gradient overlap-add runs as spec_gather8_kernel (<= 4 resolutions, <= 8 frames over a
    sample) or spec_gather_kernel (otherwise); both against the fp64 autograd oracle for these resolutions."""
    n_fft, hop, win = (list(a) for a in args)
    B, T = 2, 4096 + 77
    x, r = _signals(B, T, seed=len(n_fft) * 31 + hop[0])
    rd = r.double().squeeze(-1).clone().requires_grad_(True)
    xd = x.double().squeeze(-1)
    per = torch.stack([R.norm(R.spectral(xd, n, h, w) - R.spectral(rd, n, h, w)) / R.norm(R.spectral(xd, n, h, w))
                       for n, h, w in zip(n_fft, hop, win)], dim=-1).mean(dim=-1)
    (g_ref,) = torch.autograd.grad(per.mean(), rd)
    out = torch.empty(1, device=cuda)
    dr = torch.empty(B, T, device=cuda)
    V.spectral_loss(x.squeeze(-1).to(cuda).contiguous(), r.squeeze(-1).to(cuda).contiguous(), out, dr, None,
                    n_fft, hop, win)
    assert abs(float(out) - float(per.mean())) / float(per.mean()) < 1e-5
    err = (dr.cpu().double() - g_ref).abs().max() / g_ref.abs().max()
    assert err < 1e-4, err


@pytest.mark.parametrize("B,T", [(3, 4096 + 113), (1, 1200), (2, 8192 + 1)])
def test_pair_magnitudes_vs_oracle(cuda, B, T):
    """The target spectrograms as vqa_spectral_target writes them (the frame-pair kernel in its magnitude mode, both
    frames of a pair from one complex FFT; an odd frame count leaves the last frame unpaired), read out of the
    target buffer by its layout (per resolution: twiddles 2N | window | |S_x| (B*F, N/2 + 1), each 64-float
    aligned), against the oracle's |tf.signal.stft| at 2e-6 of the spectrum's max."""
    x, _ = _signals(B, T, seed=5 + T)
    tgt = SpectralTarget(x.to(cuda))
    buf = tgt.mags.view(torch.float32).cpu() if tgt.mags.dtype != torch.float32 else tgt.mags.cpu()
    al = lambda n: (n + 63) // 64 * 64  # noqa: E731
    o = 0
    for n_fft, hop, win in RES:
        F = 1 + (T - win) // hop
        o += al(2 * n_fft) + al(win)
        got = buf[o:o + B * F * (n_fft // 2 + 1)].double().reshape(B, F, n_fft // 2 + 1)
        o += al(B * F * (n_fft // 2 + 1))
        ref = R.spectral(x.squeeze(-1).double(), n_fft, hop, win)
        assert got.shape == ref.shape, (got.shape, ref.shape)
        err = (got - ref).abs().max() / ref.abs().max()
        assert err < 2e-6, (n_fft, float(err))
