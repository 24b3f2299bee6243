"""Conv kernel parity: libvqa (through the C-ABI) vs the CPU oracle's TF-semantics convs (fp64).

Covers every conv shape of the model (encdec.py:33,38,60,67-68,148; resnet.py:13,17) in all three
directions (forward, data-gradient, weight-gradient), with the fused ReLU / residual / ReLU'-mask flags,
fp32 (tolerance 2e-5 relative to the max magnitude) and bf16 (2e-2), plus ragged and tiny lengths.
"""
import numpy as np
import pytest
import torch

import vqa_lib as V
from oracle.vqvae_ref import conv1d as ref_conv, conv1d_transpose as ref_convT, same_pad

pytestmark = pytest.mark.gpu

TOL = {torch.float32: 2e-5, torch.bfloat16: 2.5e-2}


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / max(b.abs().max(), 1e-12))


def _q(t, dt):
    """round to the activation dtype (what the kernel sees), back to fp64 for the reference"""
    return t.to(dt).double()


CONV_CASES = [
    # (C_in, C_out, K, stride, dilation, B, T)
    (1, 32, 4, 2, 1, 2, 1024),     # first encoder down conv (generic path, fp32 waveform in)
    (1, 32, 4, 2, 1, 1, 1537),     # ... ragged: last row block partial, SAME pad on both ends
    (1, 64, 3, 1, 3, 2, 700),      # one-input-channel kernel with 64 outputs, dilated
    (32, 32, 4, 2, 1, 2, 1000),    # down conv, ragged length
    (32, 32, 4, 2, 1, 1, 513),     # odd length: SAME pads (1, 2)
    (64, 32, 4, 2, 1, 3, 512),     # level>=1 first down conv
    (32, 32, 3, 1, 1, 2, 777),     # residual conv_b
    (32, 32, 3, 1, 3, 2, 1024),
    (32, 32, 3, 1, 9, 1, 300),
    (32, 32, 3, 1, 27, 2, 2048),
    (32, 32, 3, 1, 27, 1, 40),     # dilation halo wider than the signal
    (32, 64, 3, 1, 1, 2, 515),     # encoder projection
    (64, 32, 3, 1, 1, 2, 512),     # decoder pre-conv
    (64, 1, 3, 1, 1, 2, 1024),     # decoder output conv (row-dot kernels, fp32 out)
    (64, 1, 3, 1, 1, 3, 65536),    # ... at the cfg2 chunk length
    (32, 1, 3, 1, 1, 2, 700),      # ragged tile, 32 channels
    (64, 1, 3, 1, 3, 1, 300),      # dilated taps
    (64, 1, 2, 1, 1, 2, 513),      # even kernel: SAME pads (0, 1)
    (8, 32, 3, 1, 3, 2, 256),      # generic small widths
    (32, 8, 3, 1, 1, 2, 256),
    (128, 32, 3, 1, 1, 2, 64),     # ConditionerNet pre conv (embed width 128 -> residual width 32)
    (32, 128, 3, 1, 1, 2, 300),    # 128-channel output
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv1d_fwd_bwd(cuda, case, dt):
    Cin, Cout, K, s, d, B, T = case
    g = torch.Generator().manual_seed(hash(case) % 2**31)
    x = torch.randn(B, T, Cin, generator=g, dtype=torch.float64)
    W = torch.randn(K, Cin, Cout, generator=g, dtype=torch.float64) / np.sqrt(K * Cin)
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    To, pl, _ = same_pad(T, K, s, d)
    dy = torch.randn(B, To, Cout, generator=g, dtype=torch.float64)
    xdt = torch.float32 if Cin == 1 else dt   # waveform side is fp32
    ydt = torch.float32 if Cout == 1 else dt
    flags_x = V.X_F32 if (xdt == torch.float32 and dt != torch.float32) else 0
    flags_y = V.Y_F32 if (ydt == torch.float32 and dt != torch.float32) else 0
    cd = V.dtype_code(dt)
    xq, dyq = _q(x, xdt), _q(dy, ydt)
    Wq = W.float().double()
    bq = b.float().double()
    Wd, bd = W.float().to(cuda), b.float().to(cuda)
    xd, dyd = x.to(xdt).to(cuda), dy.to(ydt).to(cuda)
    tol = TOL[dt]

    for pre_relu in (False, True):
        # forward, optional residual when shapes allow
        use_res = (Cin == Cout and s == 1)
        res = torch.randn(B, To, Cout, generator=g, dtype=torch.float64) if use_res else None
        y = torch.empty(B, To, Cout, dtype=ydt, device=cuda)
        fl = flags_x | flags_y | (V.PRE_RELU if pre_relu else 0) | (V.ADD_RESIDUAL if use_res else 0)
        V.conv1d_fwd(xd, Wd, bd, res.to(ydt).to(cuda) if use_res else None, y, B, T, To, Cin, Cout, K, s, d, pl,
                     fl, cd)
        xin = torch.relu(xq) if pre_relu else xq
        ref = ref_conv(xin, Wq, bq, s, d)
        if use_res:
            ref = _q(res, ydt) + ref
        assert _rel(y, ref) < tol, f"fwd pre_relu={pre_relu}"

    # data gradient (with ReLU' mask = x and a residual)
    if Cin > 1:
        xv = xq.clone().requires_grad_(True)
        (gx,) = torch.autograd.grad((ref_conv(xv, Wq, bq, s, d) * dyq).sum(), xv)
        resid = torch.randn(B, T, Cin, generator=g, dtype=torch.float64)
        dx = torch.empty(B, T, Cin, dtype=xdt, device=cuda)
        V.conv1d_bwd_data(dyd, Wd, xd, resid.to(xdt).to(cuda), dx, B, T, To, Cin, Cout, K, s, d, pl,
                          flags_x | flags_y | V.POST_MASK | V.ADD_RESIDUAL, cd)
        ref = _q(resid, xdt) + torch.where(xq > 0, gx, torch.zeros_like(gx))
        assert _rel(dx, ref) < tol, "bwd_data"
        dx2 = torch.empty(B, T, Cin, dtype=xdt, device=cuda)
        V.conv1d_bwd_data(dyd, Wd, None, None, dx2, B, T, To, Cin, Cout, K, s, d, pl, flags_x | flags_y, cd)
        assert _rel(dx2, gx) < tol, "bwd_data plain"

    # weight gradient (pre-ReLU on x)
    for pre_relu in (False, True):
        Wv = Wq.clone().requires_grad_(True)
        bv = bq.clone().requires_grad_(True)
        xin = torch.relu(xq) if pre_relu else xq
        gW, gb = torch.autograd.grad((ref_conv(xin, Wv, bv, s, d) * dyq).sum(), (Wv, bv))
        dW = torch.empty(K, Cin, Cout, dtype=torch.float32, device=cuda)
        db = torch.empty(Cout, dtype=torch.float32, device=cuda)
        V.conv1d_bwd_weight(xd, dyd, dW, db, B, T, To, Cin, Cout, K, s, d, pl,
                            flags_x | flags_y | (V.PRE_RELU if pre_relu else 0), cd)
        assert _rel(dW, gW) < tol * 2, f"bwd_weight dW pre_relu={pre_relu}"
        assert _rel(db, gb) < tol * 2, "bwd_weight db"

    # fused data + weight gradient (vqa_conv1d_bwd_data_weight): one kernel for the stride-1 32-channel
    # convs, the two-call fallback elsewhere; dx must equal the plain data-gradient call bit for bit
    if Cin > 1:
        for pre_relu, use_res, deferred in ((True, True, False), (True, False, True), (False, False, False)):
            Wv = Wq.clone().requires_grad_(True)
            bv = bq.clone().requires_grad_(True)
            xv = xq.clone().requires_grad_(True)
            xin = torch.relu(xv) if pre_relu else xv
            gx, gW, gb = torch.autograd.grad((ref_conv(xin, Wv, bv, s, d) * dyq).sum(), (xv, Wv, bv))
            resid = torch.randn(B, T, Cin, generator=g, dtype=torch.float64) if use_res else None
            rd = resid.to(xdt).to(cuda) if use_res else None
            dx = torch.empty(B, T, Cin, dtype=xdt, device=cuda)
            dW = torch.full((K, Cin, Cout), float("nan"), dtype=torch.float32, device=cuda)
            db = torch.full((Cout,), float("nan"), dtype=torch.float32, device=cuda)
            fl = flags_x | flags_y | (V.PRE_RELU if pre_relu else 0) | (V.ADD_RESIDUAL if use_res else 0)
            dfr = V.Deferred() if deferred else None
            V.conv1d_bwd_data_weight(dyd, Wd, xd, rd, dx, dW, db, B, T, To, Cin, Cout, K, s, d, pl, fl, cd, dfr)
            if dfr is not None:
                dfr.flush()
            ref = gx + (_q(resid, xdt) if use_res else 0)
            tag = f"fused pre_relu={pre_relu} res={use_res} deferred={deferred}"
            assert _rel(dx, ref) < tol, f"{tag}: dx"
            assert _rel(dW, gW) < tol * 2, f"{tag}: dW"
            assert _rel(db, gb) < tol * 2, f"{tag}: db"
            dx_plain = torch.empty_like(dx)
            V.conv1d_bwd_data(dyd, Wd, xd if pre_relu else None, rd, dx_plain, B, T, To, Cin, Cout, K, s, d, pl,
                              flags_x | flags_y | (V.POST_MASK if pre_relu else 0) | (V.ADD_RESIDUAL if use_res else 0),
                              cd)
            assert torch.equal(dx, dx_plain), f"{tag}: dx differs from vqa_conv1d_bwd_data"


CONVT_CASES = [
    # (C_in, C_out, B, T_in)
    (32, 32, 2, 512),
    (32, 64, 2, 300),   # last up conv maps to latent width
    (32, 32, 1, 37),
    (32, 8, 2, 128),    # generic path
    (64, 32, 2, 256),
    (32, 128, 2, 64),   # ConditionerNet last up conv (residual width 32 -> embed width 128)
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONVT_CASES)
def test_conv1d_transpose(cuda, case, dt):
    Cin, Cout, B, T = case
    K, s = 4, 2
    g = torch.Generator().manual_seed(1000 + hash(case) % 2**31)
    x = torch.randn(B, T, Cin, generator=g, dtype=torch.float64)
    W = torch.randn(K, Cout, Cin, generator=g, dtype=torch.float64) / np.sqrt(K * Cin)
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    To = s * T
    _, pl, _ = same_pad(To, K, s, 1)
    assert pl == 1
    dy = torch.randn(B, To, Cout, generator=g, dtype=torch.float64)
    cd = V.dtype_code(dt)
    xq, dyq, Wq, bq = _q(x, dt), _q(dy, dt), W.float().double(), b.float().double()
    xd, dyd, Wd, bd = x.to(dt).to(cuda), dy.to(dt).to(cuda), W.float().to(cuda), b.float().to(cuda)
    tol = TOL[dt]

    y = torch.empty(B, To, Cout, dtype=dt, device=cuda)
    V.conv1d_transpose_fwd(xd, Wd, bd, None, y, B, T, To, Cin, Cout, K, s, pl, 0, cd)
    assert _rel(y, ref_convT(xq, Wq, bq, s)) < tol, "convT fwd"

    xv = xq.clone().requires_grad_(True)
    (gx,) = torch.autograd.grad((ref_convT(xv, Wq, bq, s) * dyq).sum(), xv)
    dx = torch.empty(B, T, Cin, dtype=dt, device=cuda)
    V.conv1d_transpose_bwd_data(dyd, Wd, xd, None, dx, B, T, To, Cin, Cout, K, s, pl, V.POST_MASK, cd)
    assert _rel(dx, torch.where(xq > 0, gx, torch.zeros_like(gx))) < tol, "convT bwd_data"

    Wv, bv = Wq.clone().requires_grad_(True), bq.clone().requires_grad_(True)
    gW, gb = torch.autograd.grad((ref_convT(xq, Wv, bv, s) * dyq).sum(), (Wv, bv))
    dW = torch.empty(K, Cout, Cin, dtype=torch.float32, device=cuda)
    db = torch.empty(Cout, dtype=torch.float32, device=cuda)
    V.conv1d_transpose_bwd_weight(xd, dyd, dW, db, B, T, To, Cin, Cout, K, s, pl, 0, cd)
    assert _rel(dW, gW) < tol * 2, "convT dW"
    assert _rel(db, gb) < tol * 2, "convT db"


def test_conv_rejects_bad_args(cuda):
    x = torch.zeros(1, 16, 32, device=cuda)
    W = torch.zeros(3, 32, 32, device=cuda)
    y = torch.zeros(1, 16, 32, device=cuda)
    with pytest.raises(V.VQAError, match="T_out"):
        V.conv1d_fwd(x, W, None, None, y, 1, 16, 15, 32, 32, 3, 1, 1, 1, 0, V.F32)
    with pytest.raises(V.VQAError, match="mask"):
        V.conv1d_bwd_data(y, W, None, None, x, 1, 16, 16, 32, 32, 3, 1, 1, 1, V.POST_MASK, V.F32)
    with pytest.raises(V.VQAError, match="stride 2"):
        V.conv1d_transpose_fwd(x, W, None, None, y, 1, 16, 48, 32, 32, 3, 3, 1, 0, V.F32)
