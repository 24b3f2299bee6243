"""ConditionerNet (src/conditioner/conditioners.py:42-72) on libvqa vs the fp64 oracle (oracle/conditioner_ref.py),
at the prior's configuration (embed_width = d_model 128, residual_width 32, residual_depth 8, dilation_factor 3,
dilation_cycle 4, stride 2; Sampler.py:25, prior.py:415): forward within 1e-5 (fp32) / 2e-2 (bf16) relative,
every parameter gradient against fp64 autograd (fp32: per-tensor relative L2 <= 1e-3 — a pre-activation within
rounding of 0 can take the other ReLU branch, see test_gpu_train — and median <= 1e-5; bf16: direction and
overall magnitude, see the test), the LayerNorm and
Embedding kernels alone strictly, the Embedding gradient bit-identical to its fixed summation order, repeated
backward bitwise identical."""
import numpy as np
import pytest
import torch

import vqa_lib as V
from conditioners import ConditionerNet
from oracle import conditioner_ref as CR

pytestmark = pytest.mark.gpu

CFG = dict(bins=64, embed_width=128, residual_width=32, residual_depth=8, down_depth=3, stride=2, dilation_factor=3,
           dilation_cycle=4)


def _l2(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _net(L, dtype, cuda):
    net = ConditionerNet((L,), **CFG)
    net.build_standalone(cuda, dtype=dtype, seed=3)
    return net


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2e-2)])
def test_conditioner_forward_backward_vs_oracle(cuda, dtype, tol):
    B, L = 2, 32
    net = _net(L, dtype, cuda)
    g = torch.Generator().manual_seed(5)
    idx = torch.randint(0, CFG["bins"], (B, L), generator=g)
    st = net.store
    vals = st.values()
    p = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in vals.items()}
    want = CR.conditioner_forward(p, idx, net.name, CFG["down_depth"], CFG["stride"], CFG["residual_depth"],
                                  CFG["dilation_factor"], False, CFG["dilation_cycle"])
    y = net.forward(idx.to(cuda), save=True)
    assert tuple(y.shape) == (B, L * 8, CFG["embed_width"])
    assert _l2(y.float(), want.detach()) < tol
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    st.grad.zero_()
    net.backward(dy.to(cuda).to(dtype))
    torch.cuda.synchronize()
    grads = torch.autograd.grad((want * dy).sum(), list(p.values()))
    got = st.grads()
    errs = {k: _l2(got[k], gr) for k, gr in zip(p, grads)}
    print({k.split("/", 1)[1]: round(e, 5) for k, e in errs.items()})
    if dtype == torch.float32:
        bad = {k: e for k, e in errs.items() if not e < 1e-3}
        assert not bad, f"relative L2 over 1e-3: {bad}"
        assert np.median(list(errs.values())) < 1e-5
    else:
        # bf16 activations round every one of the 24 residual blocks' pre-activations, so ReLU masks near 0
        # differ from a wider type's and the end-to-end gradient drifts through the depth. The strict bf16 check is
        # test_conditioner_bf16_blocks_teacher_forced (every block against fp64 on its own inputs and masks);
        # here, against the SAME network run in fp32 on the GPU: the whole gradient and every tensor's direction.
        net32 = _net(L, torch.float32, cuda)
        y32 = net32.forward(idx.to(cuda), save=True)
        net32.store.grad.zero_()
        net32.backward(dy.to(cuda).float())
        torch.cuda.synchronize()
        g32 = net32.store.grads()
        errs32 = {k: _l2(got[k], g32[k]) for k in p}
        print("bf16 vs fp32 GPU:", {k.split("/", 1)[1]: round(e, 4) for k, e in errs32.items()})
        assert _l2(y.float(), y32) < 2e-2
        flat_got = np.concatenate([got[k].ravel() for k in p]).astype(np.float64)
        flat_32 = np.concatenate([g32[k].ravel() for k in p]).astype(np.float64)
        # measured: 0.19 overall; 0.2-0.3 on the embedding end, 0.01 on the LayerNorm end (24 blocks of bf16)
        assert np.linalg.norm(flat_got - flat_32) / np.linalg.norm(flat_32) < 0.25
        for k in p:
            a, b = got[k].ravel().astype(np.float64), g32[k].ravel().astype(np.float64)
            cos = float(a @ b / max(np.linalg.norm(a) * np.linalg.norm(b), 1e-30))
            assert cos >= 0.95, f"{k}: cosine {cos:.3f} vs the fp32 network"
    # the embedding gradient: rows of unused codes are exactly zero
    used = torch.zeros(CFG["bins"], dtype=torch.bool)
    used[idx.reshape(-1)] = True
    assert (got[f"{net.name}/embedding/embeddings"][~used.numpy()] == 0).all()


def test_conditioner_bf16_blocks_teacher_forced(cuda, monkeypatch):
    """Every residual block of the bf16 ConditionerNet (24 fused blocks, cyclic dilations 1, 3, 9, 27) against fp64
    autograd on the GPU's own saved input, upstream gradient and relu(h) masks: dx and all four weight gradients
    within 1e-2 relative L2 (the bf16 roundings of dh and dx). No ReLU branch can flip, so the bound is strict."""
    import resnet
    from test_gpu_resblock import block_grads_fp64
    B, L = 2, 32
    net = _net(L, torch.bfloat16, cuda)
    g = torch.Generator().manual_seed(5)
    idx = torch.randint(0, CFG["bins"], (B, L), generator=g)
    y = net.forward(idx.to(cuda), save=True)
    dy = torch.randn(y.shape, generator=g)
    log = []
    orig = resnet.ResnetConv1DBlock.backward

    def spy(self, d_y):
        x = self._saved[0]
        h, y_ = torch.empty_like(x), torch.empty_like(x)
        V.resblock_fwd(x, self.conv_a.w, self.conv_a.b, self.conv_b.w, self.conv_b.b, y_, self.dilation, h_out=h)
        rec = dict(blk=self, x=x.cpu(), h=h.cpu(), dy=d_y.cpu(),
                   W={"wa": self.conv_a.w.to(torch.bfloat16).cpu(), "ba": self.conv_a.b.cpu(),
                      "wb": self.conv_b.w.to(torch.bfloat16).cpu(), "bb": self.conv_b.b.cpu()})
        dx = orig(self, d_y)
        rec["dx"] = dx.cpu()
        log.append(rec)
        return dx

    monkeypatch.setattr(resnet.ResnetConv1DBlock, "backward", spy)
    net.store.grad.zero_()
    net.backward(dy.to(cuda).to(torch.bfloat16))
    torch.cuda.synchronize()
    monkeypatch.undo()
    assert len(log) == 24 and {r["blk"].dilation for r in log} == {1, 3, 9, 27}
    got = net.store.grads()
    for rec in log:
        blk = rec["blk"]
        want = block_grads_fp64(rec["x"], rec["dy"], rec["h"], rec["W"], blk.dilation)
        errs = {"dx": _l2(rec["dx"], want[0])}
        for k, gr, pn in zip(("wa", "ba", "wb", "bb"), want[1:], (f"{blk.conv_a.name}/kernel", f"{blk.conv_a.name}/bias",
                                                                 f"{blk.conv_b.name}/kernel", f"{blk.conv_b.name}/bias")):
            errs[k] = _l2(got[pn], gr)
        bad = {k: e for k, e in errs.items() if not e < 1e-2}
        assert not bad, f"{blk.conv_a.name} d={blk.dilation}: {bad}"


def test_conditioner_call_checks_shapes(cuda):
    net = ConditionerNet((16,), **CFG)
    out = net(np.random.default_rng(0).integers(0, CFG["bins"], (3, 16)))
    assert tuple(out.shape) == (3, 128, 128)
    with pytest.raises(ValueError, match="Upper Level Shape"):
        net(np.zeros((3, 8), np.int64))


@pytest.mark.parametrize("C,rows", [(128, 1000), (64, 77), (96, 5), (1024, 33)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_layernorm_kernels(cuda, C, rows, dtype):
    g = torch.Generator().manual_seed(C + rows)
    x = (torch.randn(rows, C, generator=g) * 3 + 1).to(dtype)
    gamma, beta = torch.randn(C, generator=g), torch.randn(C, generator=g)
    dy = torch.randn(rows, C, generator=g).to(dtype)
    xd = x.to(cuda)
    y = torch.empty_like(xd)
    V.layernorm_fwd(xd, gamma.cuda(), beta.cuda(), y, 1e-6)
    xv = x.double().requires_grad_(True)
    gv, bv = gamma.double().requires_grad_(True), beta.double().requires_grad_(True)
    want = CR.layer_norm(xv, gv, bv, 1e-6)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert _l2(y, want.detach()) < tol
    dx = torch.empty_like(xd)
    dg, db = torch.empty(C, device=cuda), torch.empty(C, device=cuda)
    V.layernorm_bwd(xd, dy.to(cuda), gamma.cuda(), dx, dg, db, 1e-6)
    gx, gg, gb = torch.autograd.grad((want * dy.double()).sum(), [xv, gv, bv])
    assert _l2(dx, gx) < tol and _l2(dg, gg) < tol and _l2(db, gb) < tol


def test_embedding_kernels_exact(cuda):
    """Gather bit-exact (fp32) / exact rounding (bf16); out-of-range index -> zero row; the backward's per-code
    sums bit-identical to the fixed summation order (tests/test_gpu_vq.py restatement) and repeatable."""
    from test_gpu_vq import _fixed_order_sums
    K, D, N = 300, 128, 5000
    g = torch.Generator().manual_seed(2)
    table = torch.randn(K, D, generator=g)
    idx = torch.randint(0, K, (N,), generator=g)
    idx[:700] = 7  # a code spanning several 64-row tiles
    idx[5] = K + 3  # out of range: zero row forward, ignored backward
    out = torch.empty(N, D, device=cuda)
    V.embedding_fwd(table.cuda(), idx.cuda(), out)
    ref = torch.zeros(N, D)
    ok = idx < K
    ref[ok] = table[idx[ok]]
    assert torch.equal(out.cpu(), ref)
    ob = torch.empty(N, D, device=cuda, dtype=torch.bfloat16)
    V.embedding_fwd(table.cuda(), idx.cuda(), ob)
    assert torch.equal(ob.cpu(), ref.to(torch.bfloat16))
    dy = torch.randn(N, D, generator=g)
    res = []
    for _ in range(2):
        dt = torch.zeros(K, D, device=cuda)
        V.embedding_bwd(dy.cuda(), idx.cuda(), dt)
        res.append(dt.cpu())
    assert torch.equal(res[0], res[1])
    want, _ = _fixed_order_sums(dy[ok].numpy(), idx[ok].numpy(), K)
    assert np.array_equal(res[0].numpy(), want)
