"""Reconstruction loss kernel (vqa_mse_loss: vqvae.py:301-307 _reconstruction_loss = mean((x - r)^2) and its
gradient 2(r - x)/n, plus an optional gradient to add) vs an fp64 restatement. The float4 kernel serves n % 4 == 0
on 16-byte aligned buffers, the scalar kernel everything else; the gradient is bitwise the same either way (the
same fp32 operations per element), the loss within fp32 summation-order rounding (1e-6 relative).
"""
import pytest
import torch

import vqa_lib as V

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [2 * 65536, 4096 + 4, 1001, 3])
@pytest.mark.parametrize("with_extra", [False, True])
def test_mse_loss_forms(cuda, n, with_extra):
    g = torch.Generator().manual_seed(n)
    x, r, e = (torch.randn(n, generator=g) for _ in range(3))
    res = []
    for off in (0, 1):  # off = 1: buffers one float past a 16-byte boundary (the scalar kernel)
        def place(t):
            buf = torch.zeros(n + 8, device=cuda)
            v = buf[off:off + n]
            v.copy_(t.to(cuda))
            return v
        xd, rd, ed, dr = place(x), place(r), place(e), place(torch.zeros(n))
        loss = torch.empty(1, device=cuda)
        V.mse_loss(xd, rd, ed if with_extra else None, dr, loss)
        res.append((float(loss), dr.cpu()))
    want = float(((r.double() - x.double()) ** 2).mean())
    gref = (2.0 / n) * (r.double() - x.double()) + (e.double() if with_extra else 0.0)
    for lo, dr in res:
        assert abs(lo - want) <= 1e-6 * want
        assert torch.allclose(dr.double(), gref, rtol=1e-6, atol=1e-9)
    assert torch.equal(res[0][1], res[1][1])
