"""Vector-quantizer kernel parity (VectorQuantizer.py:75-199) vs the CPU oracle.

Indices are compared bit-exactly on every row whose fp64 top-2 distance margin exceeds
1e-5 * |d_min|; near-tie rows are counted and must be rare. Everything else fp32 within
1e-6..1e-5 relative.
"""
import numpy as np
import pytest
import torch

import vqa_lib as V
from oracle import reset_perm
from VectorQuantizer import VectorQuantizer

pytestmark = pytest.mark.gpu


def _ref_dist(z, E):
    z = z.double()
    E = E.double()
    return (z * z).sum(1, keepdim=True) + (E * E).sum(0) - 2 * z @ E


def _margin_mask(d):
    top2 = torch.topk(d, 2, dim=1, largest=False).values
    margin = top2[:, 1] - top2[:, 0]
    return margin > 1e-5 * top2[:, 0].abs().clamp(min=1e-12)


@pytest.mark.parametrize("D,K,N", [(64, 2048, 20000), (64, 256, 2048), (8, 1024, 512), (4, 16, 1000),
                                   (16, 100, 333), (6, 50, 77)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_argmin_exact(cuda, D, K, N, dt):
    g = torch.Generator().manual_seed(D * 7 + K)
    z = torch.randn(N, D, generator=g).to(dt)
    E = (torch.rand(D, K, generator=g) - 0.5) * 0.1 + 0.05 * torch.randn(D, K, generator=g)
    zd, Ed = z.to(cuda), E.to(cuda)
    esq = torch.empty(K, device=cuda)
    V.vq_sqnorm(Ed, esq)
    idx = torch.empty(N, dtype=torch.int64, device=cuda)
    mind = torch.empty(N, device=cuda)
    V.vq_argmin(zd, Ed, esq, idx, mind)
    d = _ref_dist(z.float(), E)
    ref = d.argmin(1)
    ok = _margin_mask(d)
    got = idx.cpu()
    assert ok.float().mean() > 0.99
    assert torch.equal(got[ok], ref[ok]), f"{int((got[ok] != ref[ok]).sum())} mismatches on clear rows"
    # min distance equals the fp32 distance of the chosen code
    assert torch.allclose(mind.cpu().double(), d.gather(1, got[:, None]).squeeze(1), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("D,K,N", [(64, 2048, 262144), (64, 2048, 20000), (64, 256, 2048), (32, 1024, 777),
                                   (64, 100, 333), (32, 70, 300)])
def test_argmin_split_exact(cuda, D, K, N):
    """bf16 z on bf16 MFMA with the exact hi/mid/lo planes of E: same indices as the fp32 path and the fp64
    reference on every clear row, ragged N and K (not multiples of the 256-row / 64-code tiles)."""
    g = torch.Generator().manual_seed(D * 13 + K + N)
    z = torch.randn(N, D, generator=g).to(torch.bfloat16)
    E = (torch.rand(D, K, generator=g) - 0.5) * 0.1 + 0.05 * torch.randn(D, K, generator=g)
    zd, Ed = z.to(cuda), E.to(cuda)
    esq = torch.empty(K, device=cuda)
    V.vq_sqnorm(Ed, esq)
    E3 = torch.empty(K, 3, D, dtype=torch.bfloat16, device=cuda)
    V.vq_split_bf16x3(Ed, E3)
    # the planes reconstruct E exactly
    P = E3.float().cpu()
    assert torch.equal((P[:, 0] + P[:, 1] + P[:, 2]).t(), E)
    idx = torch.empty(N, dtype=torch.int64, device=cuda)
    mind = torch.empty(N, device=cuda)
    V.vq_argmin_split(zd, E3, esq, idx, mind)
    idx32 = torch.empty(N, dtype=torch.int64, device=cuda)
    V.vq_argmin(zd, Ed, esq, idx32)
    d = _ref_dist(z.float(), E)
    ok = _margin_mask(d)
    got = idx.cpu()
    assert ok.float().mean() > 0.99
    assert torch.equal(got[ok], d.argmin(1)[ok])
    assert (got == idx32.cpu()).float().mean() > 0.999
    assert torch.allclose(mind.cpu().double(), d.gather(1, got[:, None]).squeeze(1), rtol=1e-5, atol=1e-5)


def test_argmin_split_ties_lowest_index(cuda):
    D, K = 64, 512
    E = torch.zeros(D, K)
    E[:, 7] = 1.0
    E[:, 300] = 1.0
    z = torch.ones(40, D, dtype=torch.bfloat16)
    z[20:] = 0.0
    Ed = E.to(cuda)
    esq = torch.empty(K, device=cuda)
    V.vq_sqnorm(Ed, esq)
    E3 = torch.empty(K, 3, D, dtype=torch.bfloat16, device=cuda)
    V.vq_split_bf16x3(Ed, E3)
    idx = torch.empty(40, dtype=torch.int64, device=cuda)
    V.vq_argmin_split(z.to(cuda), E3, esq, idx)
    got = idx.cpu()
    assert (got[:20] == 7).all() and (got[20:] == 0).all()


def test_argmin_ties_lowest_index(cuda):
    D, K = 64, 512
    E = torch.zeros(D, K)
    E[:, 7] = 1.0
    E[:, 300] = 1.0     # duplicate code
    E[:, 301] = 1.0
    z = torch.ones(40, D)
    z[20:] = 0.0        # equidistant to every zero column -> lowest zero column (0)
    Ed, zd = E.cuda(), z.cuda()
    esq = torch.empty(K, device=cuda)
    V.vq_sqnorm(Ed, esq)
    idx = torch.empty(40, dtype=torch.int64, device=cuda)
    V.vq_argmin(zd, Ed, esq, idx)
    got = idx.cpu()
    assert (got[:20] == 7).all() and (got[20:] == 0).all()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_quantize_commit_stats_backward(cuda, dt):
    N, D, K, beta = 5000, 64, 256, 0.25
    g = torch.Generator().manual_seed(5)
    z = torch.randn(N, D, generator=g).to(dt)
    E = torch.randn(D, K, generator=g) * 0.3
    idx = torch.randint(0, K, (N,), generator=g)
    zd, ETd, idxd = z.cuda(), E.t().contiguous().cuda(), idx.cuda()
    q = torch.empty_like(zd)
    commit = torch.zeros(1, device=cuda)
    m_sumT = torch.zeros(K, D, device=cuda)
    n_sum = torch.zeros(K, device=cuda)
    V.vq_quantize(zd, ETd, idxd, q, commit, m_sumT, n_sum, beta)
    zf = z.double()
    qref = E.t()[idx].double()
    # straight-through value z + (q - z) computed in fp32 then stored (VectorQuantizer.py:114)
    st = (z.float() + (E.t()[idx] - z.float())).to(dt)
    assert torch.equal(q.cpu(), st)
    assert abs(float(commit) - beta * float(((qref - zf) ** 2).mean())) < 1e-5 * float(commit)
    onehot = torch.nn.functional.one_hot(idx, K).double()
    assert torch.allclose(m_sumT.cpu().double(), (zf.T @ onehot).T, rtol=1e-5, atol=1e-4)
    assert torch.equal(n_sum.cpu(), onehot.sum(0).float())
    dq = torch.randn(N, D, generator=g).to(dt)
    dz = torch.empty_like(zd)
    scale = 2 * beta / (N * D)
    V.vq_backward(dq.cuda(), zd, ETd, idxd, dz, scale)
    ref = (dq.float() + scale * (z.float() - E.t()[idx])).to(dt)
    assert torch.allclose(dz.cpu().float(), ref.float(), rtol=1e-2 if dt == torch.bfloat16 else 1e-6, atol=1e-6)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("D", [32, 64, 16])
def test_quantize_backward_vectorised_and_scalar_forms_agree(cuda, dt, D):
    """vq_quantize / vq_backward take the 8-channel vectorised kernels for D = 32 / 64 on 16-byte aligned rows
    and the scalar kernels otherwise (D = 16, or rows starting off a 16-byte boundary): the straight-through
    output and dz are bitwise the same either way (same fp32 arithmetic per element), the commitment loss
    within fp32 summation-order rounding, and both match the fp64 restatement."""
    N, K, beta = 3001, 512, 0.25
    g = torch.Generator().manual_seed(D)
    z = torch.randn(N, D, generator=g).to(dt)
    ET = torch.randn(K, D, generator=g)
    idx = torch.randint(0, K, (N,), generator=g)
    dq = torch.randn(N, D, generator=g).to(dt)
    scale = 2 * beta / (N * D)
    ETd, idxd = ET.cuda(), idx.cuda()
    res = []
    for off in (0, 1):  # off = 1: every row buffer starts one element past a 16-byte boundary
        def place(t):
            buf = torch.zeros(t.numel() + 8, dtype=t.dtype, device=cuda)
            v = buf[off:off + t.numel()].view(t.shape)
            v.copy_(t.cuda())
            return v
        zd, dqd = place(z), place(dq)
        q, dz = place(torch.zeros_like(z)), place(torch.zeros_like(z))
        commit = torch.zeros(1, device=cuda)
        V.vq_quantize(zd, ETd, idxd, q, commit, None, None, beta)
        V.vq_backward(dqd, zd, ETd, idxd, dz, scale)
        res.append((q.cpu(), dz.cpu(), float(commit)))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    qref = ET[idx].double()
    want = beta * float(((qref - z.double()) ** 2).mean())
    for r in res:
        assert abs(r[2] - want) < 1e-5 * want
    assert torch.equal(res[0][0], (z.float() + (ET[idx] - z.float())).to(dt))
    ref = (dq.float() + scale * (z.float() - ET[idx])).to(dt)
    assert torch.allclose(res[0][1].float(), ref.float(), rtol=1e-2 if dt == torch.bfloat16 else 1e-6, atol=1e-6)


@pytest.mark.parametrize("N,K", [(20000, 2048), (100, 256), (1000, 1000)])
def test_reset_rows_match_numpy_permutation(cuda, N, K):
    D = 8
    z = torch.randn(N, D).cuda()
    RT = torch.empty(K, D, device=cuda)
    counter = torch.tensor([5], dtype=torch.int64, device=cuda)
    V.vq_reset_rows(z, RT, 0, N, 3, counter, 1)
    rows = reset_perm.reset_rows(3, 5, 1, N, K)
    assert torch.equal(RT.cpu(), z.cpu()[torch.from_numpy(rows)])
    # sharded: two "ranks" each own half the rows; the sum of their partial RT is the global one
    half = N // 2
    RT0, RT1 = torch.empty_like(RT), torch.empty_like(RT)
    V.vq_reset_rows(z[:half].contiguous(), RT0, 0, N, 3, counter, 1)
    V.vq_reset_rows(z[half:].contiguous(), RT1, half, N, 3, counter, 1)
    assert torch.equal((RT0 + RT1).cpu(), RT.cpu())


def test_ema_apply_matches_reference_formula(cuda):
    D, K = 64, 512
    g = torch.Generator().manual_seed(9)
    E = (torch.rand(D, K, generator=g) - 0.5) * 0.1
    m_t = E.clone()
    N_t = torch.ones(K)
    n_sum = torch.zeros(K)
    n_sum[:100] = torch.randint(1, 50, (100,), generator=g).float()
    m_sumT = torch.randn(K, D, generator=g) * n_sum[:, None]
    RT = torch.randn(K, D, generator=g)
    Ed, ETd, mtd, Ntd = E.cuda(), E.t().contiguous().cuda(), m_t.cuda(), N_t.cuda()
    met = torch.zeros(3, device=cuda)
    ctr = torch.zeros(1, dtype=torch.int64, device=cuda)
    gam, omg = float(np.float32(0.99)), float(np.float32(1 - 0.99))
    V.vq_ema_apply(Ed, ETd, mtd, Ntd, m_sumT.cuda(), n_sum.cuda(), RT.cuda(), gam, omg, 1.0, met, ctr)
    # fp32 restatement of VectorQuantizer.py:128-145 (numpy float32, no fused multiply-add)
    f = np.float32
    Nn = f(gam) * N_t.numpy() + f(omg) * n_sum.numpy()
    mn = f(gam) * m_t.numpy() + f(omg) * m_sumT.numpy().T
    use = (Nn >= 1.0).astype(np.float32)[None, :]
    En = use * (mn / np.clip(Nn, f(1e-8), f(1e8))[None, :]) + (1 - use) * RT.numpy().T
    assert np.array_equal(Ntd.cpu().numpy(), Nn)
    assert np.array_equal(mtd.cpu().numpy(), mn)
    assert np.allclose(Ed.cpu().numpy(), En, rtol=2e-7, atol=0)
    assert torch.equal(ETd.cpu(), Ed.cpu().t())
    assert int(ctr) == 1
    p = n_sum / n_sum.sum()
    assert float(met[0]) == float((n_sum >= 1).sum())
    assert float(met[1]) == float((torch.from_numpy(Nn) >= 1).sum())
    assert abs(float(met[2]) + float((p * torch.log(p + 1e-8)).sum())) < 1e-4


@pytest.mark.parametrize("D,K", [(64, 2048), (8, 1024), (32, 70)])
def test_ema_apply_derived_state_bitwise(cuda, D, K):
    """vqa_vq_ema_apply_derived writes, in the EMA launch itself, the new codebook's |e|^2 and bf16 hi/mid/lo planes:
    bitwise what vqa_vq_sqnorm and vqa_vq_split_bf16x3 give for the updated E (the next argmin's inputs), and the
    EMA outputs bitwise those of vqa_vq_ema_apply."""
    g = torch.Generator().manual_seed(D + K)
    E = (torch.rand(D, K, generator=g) - 0.5) * 0.1
    n_sum = torch.zeros(K)
    n_sum[: K // 3] = torch.randint(1, 50, (K // 3,), generator=g).float()
    m_sumT = torch.randn(K, D, generator=g) * n_sum[:, None]
    RT = torch.randn(K, D, generator=g)
    gam, omg = float(np.float32(0.99)), float(np.float32(1 - 0.99))
    outs = []
    for derived in (False, True):
        Ed, ETd, mtd, Ntd = E.cuda(), E.t().contiguous().cuda(), E.clone().cuda(), torch.ones(K, device=cuda)
        ctr = torch.zeros(1, dtype=torch.int64, device=cuda)
        esq = torch.full((K,), float("nan"), device=cuda)
        E3 = torch.zeros(K, 3, D, dtype=torch.bfloat16, device=cuda)
        if derived:
            V.vq_ema_apply(Ed, ETd, mtd, Ntd, m_sumT.cuda(), n_sum.cuda(), RT.cuda(), gam, omg, 1.0, None, ctr,
                           esq=esq, E3=E3)
        else:
            V.vq_ema_apply(Ed, ETd, mtd, Ntd, m_sumT.cuda(), n_sum.cuda(), RT.cuda(), gam, omg, 1.0, None, ctr)
            V.vq_sqnorm(Ed, esq)
            V.vq_split_bf16x3(Ed, E3)
        torch.cuda.synchronize()
        outs.append([t.cpu() for t in (Ed, ETd, mtd, Ntd, esq, E3)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    P = outs[1][5].float()
    assert torch.equal((P[:, 0] + P[:, 1] + P[:, 2]).t(), outs[1][0])
    # |e|^2 as the sum of squares of the fp32 codebook, to fp32 rounding of a 64-term sum
    ref = (outs[1][0].double() ** 2).sum(0)
    assert torch.allclose(outs[1][4].double(), ref, rtol=1e-6, atol=0)


def test_vector_quantizer_layer_call(cuda):
    """VectorQuantizer.py:204-221 smoke: K=6, D=2 — the generic (D not MFMA-tiled) path."""
    torch.manual_seed(0)
    vq = VectorQuantizer(num_embeddings=6, embedding_dim=2, device=cuda)
    x = torch.randn(32, 100, 2, device=cuda)
    q, idx = vq(x)
    assert q.shape == x.shape and idx.shape == (3200,)
    assert torch.isfinite(vq.embeddings).all()
    assert float(vq.N_t.sum()) > 0


def _fixed_order_sums(z, idx, K, tile=64):
    """numpy float32 restatement of the deterministic EMA-sum order of vqa_vq_quantize (vqa_vq.hip): rows
    sorted by (code, row); a code's sum is sequential over its rows inside each 64-position tile of the sorted
    order; the tile partials of a code spanning tiles are summed sequentially in four contiguous quarters of its
    tile range (the first tile's partial leads quarter 0), then ((q0 + q1) + q2) + q3."""
    z = np.asarray(z, np.float32)
    order = np.argsort(idx, kind="stable")
    counts = np.bincount(idx, minlength=K)
    seg = np.concatenate([[0], np.cumsum(counts)])
    zs = z[order]
    out = np.zeros((K, z.shape[1]), np.float32)

    def seqsum(a):
        return np.cumsum(a, axis=0, dtype=np.float32)[-1]
    for k in range(K):
        S, E = int(seg[k]), int(seg[k + 1])
        if E <= S:
            continue
        ta, tb = S // tile, (E - 1) // tile
        if ta == tb:
            out[k] = seqsum(zs[S:E])
            continue
        parts = [seqsum(zs[S:(ta + 1) * tile])] + [seqsum(zs[t * tile:min(E, (t + 1) * tile)])
                                                   for t in range(ta + 1, tb + 1)]
        n = tb - ta
        per = (n + 3) // 4
        q = []
        for v in range(4):
            i0, i1 = min(n, v * per), min(n, (v + 1) * per)
            s = parts[0] if v == 0 else np.zeros(z.shape[1], np.float32)
            for t in range(i0, i1):
                s = (s + parts[1 + t]).astype(np.float32)
            q.append(s)
        out[k] = ((q[0] + q[1]) + q[2]) + q[3]
    return out, counts.astype(np.float32)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,D,K,crowd", [(20000, 64, 256, 0.0), (50000, 64, 2048, 0.7), (777, 8, 1024, 0.0),
                                         (3001, 4, 16, 0.5), (262144, 64, 2048, 0.3)])
def test_ema_sums_deterministic_fixed_order(cuda, dt, N, D, K, crowd):
    """EMA sums (VectorQuantizer.py:123-124) are deterministic: bit-identical to the numpy float32 restatement
    of their fixed summation order, bit-identical on a repeated call, counts exact; and within fp32 rounding
    of the fp64 one-hot GEMM. `crowd`: fraction of rows sent to one code (a segment spanning many tiles)."""
    g = torch.Generator().manual_seed(N + D + K)
    z = torch.randn(N, D, generator=g).to(dt)
    idx = torch.randint(0, K, (N,), generator=g)
    if crowd:
        idx[torch.rand(N, generator=g) < crowd] = 3
    zd, idxd = z.cuda(), idx.cuda()
    ETd = torch.randn(K, D, device=cuda)
    outs = []
    for _ in range(2):
        q = torch.empty_like(zd)
        commit = torch.zeros(1, device=cuda)
        m_sumT = torch.zeros(K, D, device=cuda)
        n_sum = torch.zeros(K, device=cuda)
        V.vq_quantize(zd, ETd, idxd, q, commit, m_sumT, n_sum, 0.25)
        outs.append((m_sumT.cpu().numpy(), n_sum.cpu().numpy(), float(commit)))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    assert outs[0][2] == outs[1][2]
    want, cnt = _fixed_order_sums(z.float().numpy(), idx.numpy(), K)
    assert np.array_equal(outs[0][1], cnt)
    assert np.array_equal(outs[0][0], want), f"max diff {np.abs(outs[0][0] - want).max()}"
    ref = np.zeros((K, D))
    np.add.at(ref, idx.numpy(), z.double().numpy())
    scale = np.abs(z.double().numpy()).max() * np.sqrt(cnt.max())
    assert np.abs(outs[0][0] - ref).max() <= 1e-5 * scale


@pytest.mark.parametrize("path", ["fp32", "bf16_direct", "bf16_split"])
def test_argmin_nonfinite_rows_index_zero(cuda, path):
    """A row whose distances are all NaN / +inf resolves to code 0 (tf.argmin's initial index) instead of an
    out-of-range sentinel, and the quantizer's gathers stay in bounds."""
    D, K, N = 64, 2048, 300
    g = torch.Generator().manual_seed(1)
    dt = torch.float32 if path == "fp32" else torch.bfloat16
    z = torch.randn(N, D, generator=g)
    z[5] = float("nan")
    z[17, 3] = float("inf")
    z[18, :] = float("-inf")
    z = z.to(dt)
    E = (torch.rand(D, K, generator=g) - 0.5) * 0.1
    zd, Ed = z.cuda(), E.cuda()
    esq = torch.empty(K, device=cuda)
    V.vq_sqnorm(Ed, esq)
    idx = torch.empty(N, dtype=torch.int64, device=cuda)
    mind = torch.empty(N, device=cuda)
    if path == "bf16_split":
        E3 = torch.empty(K, 3, D, dtype=torch.bfloat16, device=cuda)
        V.vq_split_bf16x3(Ed, E3)
        V.vq_argmin_split(zd, E3, esq, idx, mind)  # N small: the codebook is split across workgroups
    else:
        V.vq_argmin(zd, Ed, esq, idx, mind)
    got = idx.cpu()
    assert int(got[5]) == 0 and int(got[17]) == 0 and int(got[18]) == 0
    assert bool(((got >= 0) & (got < K)).all())
    # the reported min distance of such a row is +inf (the distance form's value: no finite distance exists)
    md = mind.cpu()
    assert all(float(md[i]) == float("inf") for i in (5, 17, 18)), md[[5, 17, 18]]
    assert bool(torch.isfinite(md[[i for i in range(N) if i not in (5, 17, 18)]]).all())
    q = torch.empty_like(zd)
    commit = torch.zeros(1, device=cuda)
    m_sumT = torch.zeros(K, D, device=cuda)
    n_sum = torch.zeros(K, device=cuda)
    V.vq_quantize(zd, Ed.t().contiguous(), idx, q, commit, m_sumT, n_sum, 0.25)
    torch.cuda.synchronize()
    assert float(n_sum.sum()) == N


def test_argmin_split_near_ties_at_large_norm(cuda):
    """Documented divergence from the reference's formula (VectorQuantizer.py:173-185 computes the fp32 distance
    (|z|^2 + |e|^2) - 2 z.e and takes its argmin): the split kernel maximises key = z.e - |e|^2 / 2 (no |z|^2 term)
    on bf16 MFMA over the exact hi/mid/lo planes of E. Rows with a large |z| (|z|^2 ~ 2.6e5) get a second code
    4e-3 (exact distance) behind their nearest one — a near tie by SURVEY.md §8c's definition (margin below
    1e-5 |d_min| ~ 2.6), where the build is not required to agree with the fp64 argmin:
      every row with a margin above the §8c bound takes the exact nearest code (as everywhere else);
      on the crafted near ties the kernel misses the exact nearest code on no more rows than the reference's own
      fp32 distance form does (a numpy restatement of its op order): the key form has no
      |z|^2 rounding (ulp 0.03 at this norm) to lose the margin in."""
    D, K, N = 64, 1024, 4096
    g = torch.Generator().manual_seed(11)
    E = (torch.rand(D, K, generator=g) - 0.5) * 0.1
    z = (torch.randn(N, D, generator=g) * 64.0).to(torch.bfloat16)  # |z|^2 ~ 2.6e5
    zf = z.double()
    Ed = E.double()
    d = (zf * zf).sum(1, keepdim=True) + (Ed * Ed).sum(0) - 2 * zf @ Ed
    best = d.argmin(1)
    for i, r in enumerate(range(0, N, 32)):  # every 32nd row: its nearest code b gets a twin c (a code of its own)
        b, c = int(best[r]), K - 1 - i
        # e_c = e_b + t u with u orthogonal to (z_r - e_b): |z_r - e_c|^2 = |z_r - e_b|^2 + t^2 |u|^2
        v = zf[r] - Ed[:, b]
        u = torch.randn(D, generator=g, dtype=torch.float64)
        u -= (u @ v) / (v @ v) * v
        u /= u.norm()
        Ed[:, c] = Ed[:, b] + 0.004 ** 0.5 * u  # exact margin 4e-3 on row r
    E = Ed.float()
    Ed = E.double()
    d = (zf * zf).sum(1, keepdim=True) + (Ed * Ed).sum(0) - 2 * zf @ Ed
    exact = d.argmin(1)
    # the reference's fp32 op order: (|z|^2 + |e|^2) - 2 z.e, each term rounded to fp32
    z32, E32 = z.float().numpy(), E.numpy()
    zz = (z32 * z32).sum(1, keepdims=True, dtype=np.float32)
    ee = (E32 * E32).sum(0, keepdims=True, dtype=np.float32)
    ref32 = torch.from_numpy(np.argmin((zz + ee) - np.float32(2.0) * (z32 @ E32), axis=1))
    Ec, zc = E.to(cuda), z.to(cuda)
    esq = torch.empty(K, device=cuda)
    V.vq_sqnorm(Ec, esq)
    E3 = torch.empty(K, 3, D, dtype=torch.bfloat16, device=cuda)
    V.vq_split_bf16x3(Ec, E3)
    idx = torch.empty(N, dtype=torch.int64, device=cuda)
    V.vq_argmin_split(zc, E3, esq, idx)
    got = idx.cpu()
    ok = _margin_mask(d)
    top2 = torch.topk(d, 2, dim=1, largest=False).values
    # the near ties the construction left (a later crafting may move an earlier pair's code again)
    rows = torch.nonzero(top2[:, 1] - top2[:, 0] < 1e-2).flatten()  # 93 (a crafted code may be a later row's b)
    assert len(rows) >= 60 and not ok[rows].any(), "near ties by the §8c bound"
    assert ok.float().mean() > 0.5  # 68 %: at |z|^2 ~ 2.6e5 the §8c bound (~2.6) is wide against K = 1024 codes
    assert torch.equal(got[ok], exact[ok]), f"{int((got[ok] != exact[ok]).sum())} rows above the §8c margin differ"
    miss_kernel = int((got[rows] != exact[rows]).sum())
    miss_ref32 = int((ref32[rows] != exact[rows]).sum())
    print(f"crafted near ties (exact margin < 1e-2, |z|^2 ~ 2.6e5): kernel misses the exact nearest code on "
          f"{miss_kernel} of {len(rows)}, the fp32 distance form on {miss_ref32}")
    assert miss_ref32 > 0, "the construction should defeat the fp32 distance form on some rows"
    assert miss_kernel <= miss_ref32, (miss_kernel, miss_ref32)
