"""Decoder-tail kernels (vqa_dtail.hip) vs the CPU oracle in fp64.

The tail is encdec.py:67-68 (the last Conv1DTranspose, K=4, stride 2, 32 -> 64 channels) followed by
encdec.py:148 (the decoder's output Conv1D, K=3, 64 -> 1), composed into one thin convolution. The oracle
runs the two layers separately (oracle/vqvae_ref.conv1d_transpose, conv1d) in fp64 and differentiates them
with autograd. Tolerances: fp32 activations 2e-5 of the output's max-abs (the composite only re-associates
the sums); bf16 activations (h rounded to bf16 on input; dh rounded on output) 1e-2 for dh and 2e-5 for y and
the parameter gradients (both are fp32 sums of the same bf16 inputs).
"""
import pytest
import torch

import vqa_lib as V
from oracle import vqvae_ref as R

pytestmark = pytest.mark.gpu


def _params(Cu, seed):
    g = torch.Generator().manual_seed(seed)
    w_up = torch.randn(4, Cu, 32, generator=g) * 0.1
    b_up = torch.randn(Cu, generator=g) * 0.1
    w_out = torch.randn(3, Cu, 1, generator=g) * 0.1
    b_out = torch.randn(1, generator=g) * 0.1
    return w_up, b_up, w_out, b_out


def _oracle(h, dy, w_up, b_up, w_out, b_out):
    hd = h.double().clone().requires_grad_(True)
    ps = [p.double().clone().requires_grad_(True) for p in (w_up, b_up, w_out, b_out)]
    u = R.conv1d_transpose(hd, ps[0], ps[1], 2)
    y = R.conv1d(u, ps[2], ps[3])
    (y * dy.double()).sum().backward()
    return y.detach(), hd.grad, [p.grad for p in ps]


def _rel(a, b):
    return float((a.double() - b).abs().max() / b.abs().max())


@pytest.mark.parametrize("B,T,Cu,dt", [(2, 64, 64, torch.float32), (3, 37, 64, torch.float32), (1, 1, 64, torch.float32),
                                       (2, 300, 48, torch.float32), (2, 64, 64, torch.bfloat16),
                                       (4, 1000, 64, torch.bfloat16),
                                       (2, 70001, 64, torch.bfloat16)])  # several grid-stride passes, ragged last
def test_forward_backward(cuda, B, T, Cu, dt):
    g = torch.Generator().manual_seed(B * 1000 + T)
    h = torch.randn(B, T, 32, generator=g).to(dt)
    dy = torch.randn(B, 2 * T, 1, generator=g)
    w_up, b_up, w_out, b_out = _params(Cu, T)
    y_ref, dh_ref, (dwu_ref, dbu_ref, dwo_ref, dbo_ref) = _oracle(h.float(), dy, w_up, b_up, w_out, b_out)

    hd = h.to(cuda)
    p = [t.to(cuda).contiguous() for t in (w_up, b_up, w_out, b_out)]
    y = torch.empty(B, 2 * T, 1, device=cuda)
    V.dtail_fwd(hd, *p, y)
    assert _rel(y.cpu(), y_ref) < 2e-5

    dh = torch.empty_like(hd)
    grads = [torch.full_like(t, float("nan")) for t in p]  # written, not accumulated
    V.dtail_bwd(dy.to(cuda), hd, *p, dh, *grads)
    assert _rel(dh.cpu().float(), dh_ref) < (1e-2 if dt == torch.bfloat16 else 2e-5)
    for got, ref in zip(grads, (dwu_ref, dbu_ref, dwo_ref, dbo_ref)):
        assert _rel(got.cpu(), ref) < 2e-5


def test_deterministic(cuda):
    B, T = 8, 4096
    g = torch.Generator().manual_seed(5)
    h = torch.randn(B, T, 32, generator=g).to(torch.bfloat16).to(cuda)
    dy = torch.randn(B, 2 * T, 1, generator=g).to(cuda)
    p = [t.to(cuda) for t in _params(64, 9)]
    outs = []
    for _ in range(2):
        dh = torch.empty_like(h)
        grads = [torch.empty_like(t) for t in p]
        V.dtail_bwd(dy, h, *p, dh, *grads)
        outs.append([dh] + grads)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_supported():
    assert V.dtail_supported(32, 64, 4, 2, 3, 1, V.BF16)
    assert not V.dtail_supported(64, 64, 4, 2, 3, 1, V.BF16)
    assert not V.dtail_supported(32, 64, 3, 2, 3, 1, V.BF16)
    assert not V.dtail_supported(32, 64, 4, 2, 3, 2, V.F32)
