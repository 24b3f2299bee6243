"""Fused residual block (vqa_resblock.hip, resnet.py:7-29 ResnetConv1DBlock) vs the unfused conv kernels and
fp64 autograd of the oracle's TF-semantics convs.

Forward: y (and relu(h)) bit-identical to the two-call unfused path (same MFMA order, same bf16 rounding of
h). Backward (h recomputed from x): dx and the four weight gradients against fp64 autograd with the ReLU
masks of the GPU's own h — relative L2 1e-5 in fp32; in bf16 against the unfused backward within 2e-2.
Ragged lengths, T shorter than a tile, every dilation of the model (1, 3, 9, 27) and the largest supported.
"""
import numpy as np
import pytest
import torch

import vqa_lib as V
from oracle.vqvae_ref import conv1d as ref_conv

pytestmark = pytest.mark.gpu

C = 32


def _l2(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(b.norm(), 1e-30))


def _block(B, T, d, seed, dt, cuda):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, T, C, generator=g)
    wa = torch.randn(3, C, C, generator=g) / np.sqrt(3 * C)
    wb = torch.randn(3, C, C, generator=g) / np.sqrt(3 * C)
    ba = 0.1 * torch.randn(C, generator=g)
    bb = 0.1 * torch.randn(C, generator=g)
    dy = torch.randn(B, T, C, generator=g)
    to = lambda t, tdt=torch.float32: t.to(tdt).to(cuda).contiguous()  # noqa: E731
    return dict(x=to(x, dt), dy=to(dy, dt), wa=to(wa), wb=to(wb), ba=to(ba), bb=to(bb))


def _unfused_fwd(p, d):
    x = p["x"]
    B, T, _ = x.shape
    cd = V.dtype_code(x.dtype)
    h = torch.empty_like(x)
    y = torch.empty_like(x)
    V.conv1d_fwd(x, p["wa"], p["ba"], None, h, B, T, T, C, C, 3, 1, d, d, V.PRE_RELU, cd)
    V.conv1d_fwd(h, p["wb"], p["bb"], x, y, B, T, T, C, C, 3, 1, 1, 1, V.PRE_RELU | V.ADD_RESIDUAL, cd)
    return h, y


def _fused_fwd(p, d):
    x = p["x"]
    y, h = torch.empty_like(x), torch.empty_like(x)
    V.resblock_fwd(x, p["wa"], p["ba"], p["wb"], p["bb"], y, d, h_out=h)
    return h, y


def _fused_bwd(p, d, deferred=False):
    x = p["x"]
    dx = torch.empty_like(x)
    g = {k: torch.full(s, float("nan"), device=x.device) for k, s in
         (("wa", (3, C, C)), ("ba", (C,)), ("wb", (3, C, C)), ("bb", (C,)))}
    dfr = V.Deferred() if deferred else None
    V.resblock_bwd(p["dy"], x, p["wa"], p["ba"], p["wb"], p["bb"], dx, g["wa"], g["ba"], g["wb"], g["bb"], d, dfr)
    if dfr is not None:
        dfr.flush()
    return dx, g


CASES = [(2, 1000, 1), (2, 1000, 3), (1, 777, 9), (2, 2048, 27), (1, 40, 27), (3, 129, 32), (1, 300, 2)]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,T,d", CASES)
def test_forward_bitwise_vs_unfused(cuda, B, T, d, dt):
    p = _block(B, T, d, seed=B * 1000 + T + d, dt=dt, cuda=cuda)
    h0, y0 = _unfused_fwd(p, d)
    h1, y1 = _fused_fwd(p, d)
    assert torch.equal(y1, y0)
    assert torch.equal(h1, torch.relu(h0))


@pytest.mark.parametrize("B,T,d", CASES)
def test_backward_fp32_vs_autograd(cuda, B, T, d):
    p = _block(B, T, d, seed=7 * T + d, dt=torch.float32, cuda=cuda)
    h, _ = _fused_fwd(p, d)  # relu(h) exactly as the backward recomputes it: its masks
    dx, g = _fused_bwd(p, d)
    cpu = {k: v.double().cpu() for k, v in p.items()}
    W = {k: cpu[k].clone().requires_grad_(True) for k in ("wa", "ba", "wb", "bb")}
    xv = cpu["x"].clone().requires_grad_(True)
    hh = ref_conv(xv * (cpu["x"] > 0), W["wa"], W["ba"], 1, d)
    y = xv + ref_conv(hh * (h.double().cpu() > 0), W["wb"], W["bb"], 1, 1)
    grads = torch.autograd.grad((y * cpu["dy"]).sum(), [xv] + [W[k] for k in ("wa", "ba", "wb", "bb")])
    assert _l2(dx, grads[0]) < 1e-5
    for k, gr in zip(("wa", "ba", "wb", "bb"), grads[1:]):
        assert _l2(g[k], gr) < 1e-5, k


@pytest.mark.parametrize("B,T,d", [(2, 1000, 1), (2, 2048, 27), (1, 40, 27), (4, 4096, 9)])
def test_backward_bf16_vs_unfused(cuda, B, T, d):
    p = _block(B, T, d, seed=3 * T + d, dt=torch.bfloat16, cuda=cuda)
    x, dy = p["x"], p["dy"]
    cd = V.BF16
    h, _ = _unfused_fwd(p, d)
    dh = torch.empty_like(x)
    dx0 = torch.empty_like(x)
    ref = {k: torch.empty(s, device=cuda) for k, s in (("wa", (3, C, C)), ("ba", (C,)), ("wb", (3, C, C)), ("bb", (C,)))}
    V.conv1d_bwd_data_weight(dy, p["wb"], h, None, dh, ref["wb"], ref["bb"], B, T, T, C, C, 3, 1, 1, 1, V.PRE_RELU, cd)
    V.conv1d_bwd_data_weight(dh, p["wa"], x, dy, dx0, ref["wa"], ref["ba"], B, T, T, C, C, 3, 1, d, d,
                             V.PRE_RELU | V.ADD_RESIDUAL, cd)
    dx, g = _fused_bwd(p, d)
    assert _l2(dx, dx0) < 2e-2
    for k in ref:
        assert _l2(g[k], ref[k]) < 2e-2, k


def test_backward_deterministic_and_deferred(cuda):
    p = _block(4, 3000, 9, seed=5, dt=torch.bfloat16, cuda=cuda)
    dx1, g1 = _fused_bwd(p, 9)
    dx2, g2 = _fused_bwd(p, 9, deferred=True)
    assert torch.equal(dx1, dx2)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k


def _unfused_bwd(p, d, h):
    x, dy = p["x"], p["dy"]
    B, T, _ = x.shape
    cd = V.dtype_code(x.dtype)
    dh, dx0 = torch.empty_like(x), torch.empty_like(x)
    ref = {k: torch.empty(s, device=x.device) for k, s in (("wa", (3, C, C)), ("ba", (C,)), ("wb", (3, C, C)),
                                                              ("bb", (C,)))}
    V.conv1d_bwd_data_weight(dy, p["wb"], h, None, dh, ref["wb"], ref["bb"], B, T, T, C, C, 3, 1, 1, 1, V.PRE_RELU, cd)
    V.conv1d_bwd_data_weight(dh, p["wa"], x, dy, dx0, ref["wa"], ref["ba"], B, T, T, C, C, 3, 1, d, d,
                             V.PRE_RELU | V.ADD_RESIDUAL, cd)
    return dx0, ref


def block_grads_fp64(x, dy, h_gpu, W, d):
    """fp64 autograd of resnet.py:7-29 on the GPU's own bf16 inputs, with the ReLU' masks of the GPU's relu(h)
    (the weights as the kernels use them: bf16-rounded kernels, fp32 biases). -> (dx, dW_a, db_a, dW_b, db_b)."""
    x, dy = x.double().cpu(), dy.double().cpu()
    Wv = {k: W[k].double().cpu().clone().requires_grad_(True) for k in ("wa", "ba", "wb", "bb")}
    xv = x.clone().requires_grad_(True)
    hh = ref_conv(xv * (x > 0), Wv["wa"], Wv["ba"], 1, d)
    y = xv + ref_conv(hh * (h_gpu.double().cpu() > 0), Wv["wb"], Wv["bb"], 1, 1)
    return torch.autograd.grad((y * dy).sum(), [xv] + [Wv[k] for k in ("wa", "ba", "wb", "bb")])


def bf16_weights(p):
    """the kernels stage the fp32 conv kernels as bf16 MFMA operands; biases stay fp32"""
    return {"wa": p["wa"].to(torch.bfloat16), "ba": p["ba"], "wb": p["wb"].to(torch.bfloat16), "bb": p["bb"]}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("T,d", [(32768, 27), (32768, 1), (8192, 9), (512, 3)])
def test_full_size_cfg2(cuda, T, d):
    """cfg2 shapes (B = 32, bf16; T = 32768 is level 0's first stack, 512 level 2's last): forward
    bit-identical to the unfused path; backward (dx and all four weight gradients, through the persistent
    grid and the partial-row reduction at full size) against fp64 autograd of the block on the same bf16 inputs
    (the GPU's relu(h) masks; bf16 kernels) within 1e-2 relative L2 — the bf16 roundings of dh and dx — and
    against the unfused HIP backward within the bf16 bound."""
    B = 32
    p = _block(B, T, d, seed=11 + d, dt=torch.bfloat16, cuda=cuda)
    h0, y0 = _unfused_fwd(p, d)
    h1, y1 = _fused_fwd(p, d)
    assert torch.equal(y1, y0)
    dx, g = _fused_bwd(p, d)
    want = block_grads_fp64(p["x"], p["dy"], h1, bf16_weights(p), d)
    errs = {"dx": _l2(dx, want[0])}
    errs.update({k: _l2(g[k], gr) for k, gr in zip(("wa", "ba", "wb", "bb"), want[1:])})
    print(f"T={T} d={d} fp64 relative L2: " + ", ".join(f"{k} {e:.2e}" for k, e in errs.items()))
    for k, e in errs.items():
        assert e < 1e-2, f"{k} vs fp64: {e:.3e}"
    dx0, ref = _unfused_bwd(p, d, h0)
    assert _l2(dx, dx0) < 2e-2
    for k in ref:
        assert _l2(g[k], ref[k]) < 2e-2, k


def test_unsupported(cuda):
    assert not V.resblock_supported(64, 1, V.BF16)
    assert not V.resblock_supported(32, 33, V.BF16)
    assert V.resblock_supported(32, 27, V.BF16) and V.resblock_supported(32, 27, V.F32)
