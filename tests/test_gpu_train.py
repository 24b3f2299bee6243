"""End-to-end VQVAE.train_step parity (vqvae.py:111-146) vs the CPU oracle (fp64), plus the reference's
other entry points (test_step, call, encode, decode) and hipGraph replay.

fp32 model, end to end against the fp64 oracle: per-level losses rel <= 1e-5; the median over tensors of
the max-norm gradient error <= 5e-4; every tensor's relative L2 gradient error <= 1e-2. The per-tensor
bound has to be loose: a pre-activation within fp32 rounding of 0 takes the other ReLU branch in fp64,
and that one element propagates to every earlier layer (measured on cfg1: one such element in
enc0/blk0/res2/rb1 gives 2.7e-3 there while every other block is at 1e-7; on cfg2_short step 1 the worst
tensor reached 5.7e-3 while a level without a flip stays at 1e-7). The strict check is
test_every_conv_call_teacher_forced / test_resblock_backward_teacher_forced: every conv call (and every
residual block) of a real step against fp64 autograd on the GPU's own inputs and ReLU masks — no branch
can flip; bound 1e-5 relative L2 (fp32 accumulation over up to ~2^17 rows; measured <= 2.3e-6).
Each step starts the oracle from the GPU model's state (weights, Adam moments, codebook state), so the
second step is held to the same bounds as the first; the GPU's Adam update is checked against keras_adam
in fp64 on the GPU's own gradients (rel 1e-6). Codebooks after two EMA steps: relative L2 <= 1e-3; usage counts N_t equal on >= 99 %
of codes (a code can move only when a row sits on a near-tie). bf16 model (cfg1 and the
benched cfg2 at B = 32, T = 65536): losses rel <= 2e-2, code-index agreement >= 99 %;
cfg1 gradient relative L2 <= 0.15 per tensor.
"""
import numpy as np
import pytest
import torch

from oracle import vqvae_ref as R
from vqvae import VQVAE

pytestmark = pytest.mark.gpu

CONFIGS = {
    # tiny: N < K on both levels (VectorQuantizer._tile path), generic + MFMA kernels, D=8
    "tiny": dict(cfg=R.RefConfig(input_len=2048, levels=2, latent_dim=8, down_depth=[2, 1], strides=[2, 2],
                                 num_embeddings=1024, residual_width=32, residual_depth=2, dilation_factor=3), B=1),
    # BASELINE config 1: 1 level, K=256, B=4, T=4096
    "cfg1": dict(cfg=R.RefConfig(input_len=4096, levels=1, latent_dim=64, down_depth=[3], strides=[2],
                                 num_embeddings=256, residual_width=32, residual_depth=4, dilation_factor=3), B=4),
    # BASELINE config 2 architecture on a shorter chunk (3 levels, hops 8/32/128, K=2048)
    "cfg2_short": dict(cfg=R.RefConfig(input_len=8192, levels=3, latent_dim=64, down_depth=[3, 2, 2],
                                       strides=[2, 2, 2], num_embeddings=2048, residual_width=32, residual_depth=4,
                                       dilation_factor=3), B=2),
}


def _model(cfg, B, dtype, params, vq):
    m = VQVAE((cfg.input_len, 1), cfg.levels, cfg.latent_dim, cfg.down_depth, cfg.strides,
              num_embeddings=cfg.num_embeddings, residual_width=cfg.residual_width,
              residual_depth=cfg.residual_depth, dilation_factor=cfg.dilation_factor, dtype=dtype, device="cuda:0")
    m.set_weights(params)
    m.set_vq_state(vq)
    m.compile()
    return m


def out_idx(ref, level):
    """The oracle's own indices of its last step at `level`."""
    return ref.last["infos"][level]["idx"]


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-12))


def _l2(a, b):
    return float(np.linalg.norm((np.asarray(a, np.float64) - b).ravel()) / max(np.linalg.norm(np.ravel(b)), 1e-30))


def _check_grads(grads, ref_grads, l2_tol, med_tol, tag):
    maxrel = {n: _rel(grads[n], g.numpy()) for n, g in ref_grads.items()}
    l2 = {n: _l2(grads[n], g.numpy()) for n, g in ref_grads.items()}
    for n in l2:
        assert l2[n] < l2_tol, f"{tag}: grad {n} relative L2 {l2[n]:.3e}"
    med = float(np.median(list(maxrel.values())))
    assert med < med_tol, f"{tag}: median max-norm grad error {med:.3e}"


def _sync_oracle(ref, m):
    """Teacher-force the oracle onto the GPU model's state: weights, Adam moments, codebook state."""
    sd = m.state_dict()
    dt = ref.dtype
    flat = sd["weights"].to(dt)
    am = sd.get("adam_m")
    av = sd.get("adam_v")
    for n in ref.names:
        off, shape = m.store.offsets[n]
        cnt = int(np.prod(shape))
        ref.p[n] = flat[off:off + cnt].reshape(shape).clone().requires_grad_(True)
        if am is not None:
            ref.adam_m[n] = am[off:off + cnt].to(dt).reshape(shape).clone()
            ref.adam_v[n] = av[off:off + cnt].to(dt).reshape(shape).clone()
    for l, st in enumerate(sd["vq"]):
        ref.vq[l] = {k: torch.tensor(np.asarray(st[k]), dtype=dt) for k in ("embeddings", "m_t", "N_t")}
        ref.vq[l]["calls"] = int(st["calls"])


def _check_adam(m, before, t):
    """The GPU's Adam step on its own gradients vs keras_adam in fp64 (TF ApplyAdam form)."""
    after = m.state_dict()
    g = m.store.grad[:m.store.size].detach().cpu().double()
    w0 = before["weights"].double()
    m0 = before["adam_m"].double() if "adam_m" in before else torch.zeros_like(w0)
    v0 = before["adam_v"].double() if "adam_v" in before else torch.zeros_like(w0)
    w, mm, vv = R.keras_adam(w0, g, m0, v0, t)
    scale = {"w": w0.abs() + 1e-2, "m": mm.abs() + g.abs() + m0.abs(), "v": vv + g * g + v0}
    for got, want, tag in ((after["weights"], w, "w"), (after["adam_m"], mm, "m"), (after["adam_v"], vv, "v")):
        err = (got.double() - want).abs()
        # fp32 arithmetic: a few ulp of the operands (w: of |w| and of the 1e-3-sized update)
        assert bool((err <= 1e-6 * scale[tag] + 1e-30).all()), f"adam step {t} {tag}: max err {float(err.max()):.3e}"


def _capture_vq(monkeypatch):
    """Record every VectorQuantizer.forward of a step: the level, the z it quantised, the codebook it used
    and the indices it chose (host copies)."""
    import VectorQuantizer as VQ
    log = []
    orig = VQ.VectorQuantizer.forward

    def f(self, z, *a, **kw):
        E = self.embeddings.detach().double().cpu()
        q, idx = orig(self, z, *a, **kw)
        log.append({"level": self.level, "z": z.detach().reshape(-1, self.embedding_dim).double().cpu(), "E": E,
                    "idx": idx.detach().cpu()})
        return q, idx
    monkeypatch.setattr(VQ.VectorQuantizer, "forward", f)
    return log


def _check_indices_exact(rec, tag, margin=1e-5):
    """VectorQuantizer.py:173-185 on the GPU's own z and codebook: the fp64 distances' argmin must equal the
    GPU's index on every row whose top-2 margin exceeds margin*|d_min| (near-ties counted and reported)."""
    z, E = rec["z"], rec["E"]
    d = (z * z).sum(1, keepdim=True) + (E * E).sum(0) - 2 * z @ E
    top2 = torch.topk(d, 2, dim=1, largest=False).values
    clear = (top2[:, 1] - top2[:, 0]) > margin * top2[:, 0].abs().clamp(min=1e-30)
    want = d.argmin(1)
    bad = int((rec["idx"][clear] != want[clear]).sum())
    ties = int((~clear).sum())
    print(f"{tag} level {rec['level']}: {len(want)} rows, {ties} near-ties (margin <= {margin:g}), "
          f"{int((rec['idx'] != want).sum())} differ in total")
    assert bad == 0, f"{tag} level {rec['level']}: {bad} indices differ on clear-margin rows"
    return clear, want


@pytest.mark.parametrize("name", list(CONFIGS))
def test_train_step_fp32_matches_oracle(cuda, monkeypatch, name):
    c = CONFIGS[name]
    cfg, B = c["cfg"], c["B"]
    params, vq = R.init_params(cfg, 1), R.init_vq_state(cfg, 2)
    ref = R.RefVQVAE(cfg, params, vq, dtype=torch.float64)
    m = _model(cfg, B, "fp32", params, vq)
    x0 = R.synthetic_batch(B, cfg.input_len, seed=11)
    x1 = R.synthetic_batch(B, cfg.input_len, seed=12)
    hist = []
    for step, x in enumerate((x0, x1)):
        # every step starts the oracle from the GPU's state, so step 1 is checked as strictly as step 0
        # (free-running, Adam turns fp32 rounding in near-zero gradients into +-lr weight moves)
        _sync_oracle(ref, m)
        before = m.state_dict()
        out = ref.train_step(x)
        hist.append(out)
        vqlog = _capture_vq(monkeypatch)
        res = {k: float(v) for k, v in m.train_step(x).items()}
        torch.cuda.synchronize()
        monkeypatch.undo()
        assert [r["level"] for r in vqlog] == list(range(cfg.levels))
        for rec in vqlog:  # end-to-end index exactness on the GPU's own z
            _check_indices_exact(rec, f"{name} step {step}")
        for k in res:
            want = float(np.mean([h[k] for h in hist]))
            tol = 1e-5 if "usage" not in k and "entropy" not in k else 2e-2
            assert abs(res[k] - want) <= tol * max(abs(want), 1e-3), f"step {step} {k}: gpu {res[k]} oracle {want}"
        _check_grads(m.store.grads(), ref.last["grads"], 1e-2, 5e-4, f"step {step}")
        _check_adam(m, before, step + 1)
    ovq = ref.state_numpy()[1]
    for l, st in enumerate(m.get_vq_state()):
        o = ovq[l]
        same = np.isclose(st["N_t"], o["N_t"], rtol=1e-6, atol=1e-6)
        assert same.mean() >= 0.99, f"level {l}: N_t differs on {(~same).sum()} codes"
        good = np.where(same)[0]
        assert _l2(st["m_t"][:, good], o["m_t"][:, good]) < 1e-3
        assert _l2(st["embeddings"][:, good], o["embeddings"][:, good]) < 1e-3
        assert st["calls"] == o["calls"] == 2


def test_train_step_bf16_tracks_oracle(cuda, monkeypatch):
    c = CONFIGS["cfg1"]
    cfg, B = c["cfg"], c["B"]
    params, vq = R.init_params(cfg, 1), R.init_vq_state(cfg, 2)
    ref = R.RefVQVAE(cfg, params, vq, dtype=torch.float64)
    m = _model(cfg, B, "bf16", params, vq)
    x = R.synthetic_batch(B, cfg.input_len, seed=11)
    out = ref.train_step(x)
    vqlog = _capture_vq(monkeypatch)
    res = {k: float(v) for k, v in m.train_step(x).items()}
    monkeypatch.undo()
    for k in ("loss", "recon_loss", "spectral_loss", "vqvae_loss"):  # SURVEY.md §8c bf16 bound
        assert abs(res[k] - out[k]) <= 2e-2 * abs(out[k]), f"{k}: gpu {res[k]} oracle {out[k]}"
    for rec in vqlog:
        agree = float((rec["idx"] == out_idx(ref, rec["level"])).double().mean())
        assert agree >= 0.99, f"bf16 index agreement with the oracle {agree:.4f}"
    _check_grads(m.store.grads(), ref.last["grads"], 0.15, 0.15, "bf16")


CFG2 = R.RefConfig(input_len=65536, levels=3, latent_dim=64, down_depth=[3, 2, 2], strides=[2, 2, 2],
                   num_embeddings=2048, residual_width=32, residual_depth=4, dilation_factor=3)


def _oracle_level_losses(ref, x, chunk=8):
    """Per level (recon, commit, spectral) of the oracle's forward (no EMA) over the whole batch. Every loss is
    a mean over equal-size items, so chunked item means average to the batch mean."""
    out = np.zeros((ref.cfg.levels, 3))
    n = 0
    with torch.no_grad():
        for i in range(0, x.shape[0], chunk):
            xc = torch.as_tensor(x[i:i + chunk], dtype=ref.dtype)
            for l in range(ref.cfg.levels):
                inf = ref.level_forward(xc, l, training=False)
                out[l] += [float(inf["recon_loss"]), float(inf["commit"]), float(inf["spectral_loss"])]
            n += 1
    return out / n


@pytest.mark.timeout(900)
def test_train_step_bf16_cfg2_full_size(cuda, monkeypatch):
    """The benched workload itself (BASELINE config 2: 3 levels, K = 2048, B = 32, T = 65536, bf16), two
    train steps with the bench's synthetic batches. Each step: per-level recon / commitment / spectral losses
    and the total within SURVEY.md §8c's bf16 bound (2e-2 relative) of the oracle (fp32, reference op
    sequence) run on the GPU model's weights and codebooks over all 32 items; per level, the GPU's code
    indices equal the fp64 argmin on its own z on every clear-margin row, and agree on >= 99 % of rows."""
    from data_utils import synthetic_batch
    cfg, B = CFG2, 32
    params, vq = R.init_params(cfg, 1), R.init_vq_state(cfg, 2)
    m = _model(cfg, B, "bf16", params, vq)
    ref = R.RefVQVAE(cfg, params, vq, dtype=torch.float32)
    for step in range(2):
        x = synthetic_batch(B, cfg.input_len, seed=1234 + 7919 * step)
        _sync_oracle(ref, m)
        want = _oracle_level_losses(ref, x)
        vqlog = _capture_vq(monkeypatch)
        m.train_step(x)
        torch.cuda.synchronize()
        monkeypatch.undo()
        got = m.loss_slots.detach().cpu().double().numpy()  # this step's (recon, commit, spectral) per level
        for l in range(cfg.levels):
            for j, k in enumerate(("recon", "commit", "spectral")):
                rel = abs(got[l, j] - want[l, j]) / abs(want[l, j])
                print(f"step {step} level {l} {k}: gpu {got[l, j]:.6g} oracle {want[l, j]:.6g} rel {rel:.2e}")
                assert rel <= 2e-2, f"step {step} level {l} {k}"
        assert abs(got.sum() - want.sum()) <= 2e-2 * abs(want.sum())
        for rec in vqlog:
            clear, fp64_idx = _check_indices_exact(rec, f"cfg2 bf16 step {step}")
            agree = float((rec["idx"] == fp64_idx).double().mean())
            assert agree >= 0.99, f"level {rec['level']}: index agreement {agree:.4f}"


@pytest.mark.timeout(900)
def test_bf16_cfg2_full_size_level2_blocks_teacher_forced(cuda, monkeypatch):
    """The benched bf16 step (B = 32, T = 65536): every residual block of level 2 (56 fused blocks, T = 32768 down
    to 512) checked against fp64 autograd on the GPU's own saved input, upstream gradient and relu(h) masks
    (tests/test_gpu_resblock.block_grads_fp64): dx on items 0-1 of every block, and dx plus all four weight
    gradients over the whole batch for the blocks at T <= 2048 (the weight gradients sum over items, and the
    level's deferred partial reductions have run by the end of the step). Bound 1e-2 relative L2 (bf16 rounding
    of dh / dx)."""
    import resnet
    import vqa_lib as V
    from data_utils import synthetic_batch
    from test_gpu_resblock import block_grads_fp64
    cfg, B = CFG2, 32
    m = _model(cfg, B, "bf16", R.init_params(cfg, 1), R.init_vq_state(cfg, 2))
    log = []
    orig = resnet.ResnetConv1DBlock.backward

    def spy(self, dy):
        name = self.conv_a.name
        if not name.startswith(("enc2/", "dec2/")):
            return orig(self, dy)
        x = self._saved[0]
        full = x.shape[1] <= 2048
        xs = x if full else x[:2].contiguous()
        h, y_ = torch.empty_like(xs), torch.empty_like(xs)  # relu(h) exactly as the backward recomputes it
        V.resblock_fwd(xs, self.conv_a.w, self.conv_a.b, self.conv_b.w, self.conv_b.b, y_, self.dilation, h_out=h)
        rec = dict(blk=self, full=full, x=xs.cpu(), h=h.cpu(), dy=(dy if full else dy[:2]).cpu(),
                   W={"wa": self.conv_a.w.to(torch.bfloat16).cpu(), "ba": self.conv_a.b.cpu(),
                      "wb": self.conv_b.w.to(torch.bfloat16).cpu(), "bb": self.conv_b.b.cpu()})
        dx = orig(self, dy)
        rec["dx"] = (dx if full else dx[:2]).cpu()
        log.append(rec)
        return dx

    monkeypatch.setattr(resnet.ResnetConv1DBlock, "backward", spy)
    m.train_step(synthetic_batch(B, cfg.input_len, seed=1234))
    torch.cuda.synchronize()
    monkeypatch.undo()
    assert len(log) == 56
    g = m.store.grads()
    worst = {}
    for rec in log:
        blk = rec["blk"]
        want = block_grads_fp64(rec["x"], rec["dy"], rec["h"], rec["W"], blk.dilation)
        errs = {"dx": _l2(rec["dx"].double().numpy(), want[0].numpy())}
        if rec["full"]:
            for k, gr, pn in zip(("wa", "ba", "wb", "bb"), want[1:],
                                 (f"{blk.conv_a.name}/kernel", f"{blk.conv_a.name}/bias", f"{blk.conv_b.name}/kernel",
                                  f"{blk.conv_b.name}/bias")):
                errs[k] = _l2(g[pn], gr.numpy())
        for k, e in errs.items():
            worst[k] = max(worst.get(k, 0.0), e)
            assert e < 1e-2, f"{blk.conv_a.name} (T={rec['x'].shape[1]}, d={blk.dilation}) {k}: {e:.3e}"
    print("level-2 blocks vs fp64, worst relative L2:", {k: f"{v:.2e}" for k, v in worst.items()})


def test_graph_replay_matches_eager(cuda):
    c = CONFIGS["cfg1"]
    cfg, B = c["cfg"], c["B"]
    params, vq = R.init_params(cfg, 1), R.init_vq_state(cfg, 2)
    xs = [R.synthetic_batch(B, cfg.input_len, seed=20 + i) for i in range(5)]
    a = _model(cfg, B, "bf16", params, vq)
    for x in xs:
        a.train_step(x)
    b = _model(cfg, B, "bf16", params, vq)
    b.capture_train_step(xs[0], warmup=2)   # two real eager steps on xs[0]
    b.set_weights(params)                    # restart from the same state, then replay
    b.set_vq_state(vq)
    b.load_state_dict({**b.state_dict(), "adam_m": torch.zeros_like(b.optimizer.m).cpu(),
                       "adam_v": torch.zeros_like(b.optimizer.v).cpu(), "iterations": 0})
    for x in xs:
        b.train_step(x)                      # graph replays
    torch.cuda.synchronize()
    # the same kernels in the same order from the same state: bitwise equal
    assert torch.equal(a.store.flat, b.store.flat)
    for sa, sb in zip(a.get_vq_state(), b.get_vq_state()):
        assert sa["calls"] == sb["calls"]
        for k in ("embeddings", "m_t", "N_t"):
            assert np.array_equal(sa[k], sb[k]), k


def test_call_encode_decode_test_step(cuda):
    c = CONFIGS["tiny"]
    cfg, B = c["cfg"], c["B"]
    params, vq = R.init_params(cfg, 1), R.init_vq_state(cfg, 2)
    ref = R.RefVQVAE(cfg, params, vq, dtype=torch.float64)
    m = _model(cfg, B, "fp32", params, vq)
    x = R.synthetic_batch(B, cfg.input_len, seed=3)
    # call(training=False): no EMA
    recons, losses = m(x, training=False)
    rr, rl = ref.call(x, training=False)
    for l in range(cfg.levels):
        assert _rel(recons[l].cpu().numpy(), rr[l].numpy()) < 1e-4
        assert abs(float(losses["level_losses"][l]) - float(rl["level_losses"][l])) < 1e-5 * abs(float(rl["level_losses"][l]))
    assert all(st["calls"] == 0 for st in m.get_vq_state())
    # encode / decode: every clear-margin row's code equals the fp64 argmin on the GPU's own z (vqvae.py:208-219,
    # VectorQuantizer.py:170-186), and >= 99 % of all rows agree with the oracle's own encode
    import VectorQuantizer as VQ
    seen = []
    orig_gci = VQ.VectorQuantizer.get_code_indices

    def spy_gci(self, flat):
        idx = orig_gci(self, flat)
        seen.append({"level": self.level, "z": flat.detach().double().cpu(),
                     "E": self.embeddings.detach().double().cpu(), "idx": idx.detach().cpu()})
        return idx
    VQ.VectorQuantizer.get_code_indices = spy_gci
    try:
        codes = m.encode(x)
    finally:
        VQ.VectorQuantizer.get_code_indices = orig_gci
    assert [r["level"] for r in seen] == list(range(cfg.levels))
    for rec in seen:
        _check_indices_exact(rec, "encode")
    rcodes = ref.encode(x)
    for l in range(cfg.levels):
        assert codes[l].shape == rcodes[l].shape
        assert (codes[l].cpu() == rcodes[l]).float().mean() > 0.99
        dec = m.decode(codes[l], level=l)
        assert _rel(dec.cpu().numpy(), ref.decode(codes[l].cpu(), level=l).numpy()) < 1e-4
    # test_step runs the EMA (reference quirk) and returns metrics
    res = {k: float(v) for k, v in m.test_step(x).items()}
    out = ref.test_step(x)
    assert abs(res["loss"] - out["loss"]) < 1e-5 * abs(out["loss"])
    assert all(st["calls"] == 1 for st in m.get_vq_state())


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_checkpoint_resume_bitwise(cuda, tmp_path, dtype):
    """Resume from a checkpoint file reproduces the uninterrupted run bit for bit: weights, Adam state,
    codebooks (E, m_t, N_t, reset counter) and metrics. Holds because every reduction of the step runs in a
    fixed order (the EMA sums included). The file loads with torch.load(weights_only=True)."""
    c = CONFIGS["cfg1"]
    cfg, B = c["cfg"], c["B"]
    params, vq = R.init_params(cfg, 1), R.init_vq_state(cfg, 2)
    xs = [R.synthetic_batch(B, cfg.input_len, seed=40 + i) for i in range(3)]
    a = _model(cfg, B, dtype, params, vq)
    a.train_step(xs[0])
    path = str(tmp_path / "ckpt.pt")
    a.save(path)
    ck = torch.load(path, weights_only=True)
    assert ck["format"] == "vqa-vqvae/2" and int(ck["iterations"]) == 1
    # the same state written as a format-/1 file in the packed layout of the first releases (no gaps) loads by
    # name into the aligned layout
    st = a.store
    pack = lambda flat: torch.cat([flat[o:o + int(np.prod(sh))] for _, (o, sh) in st.offsets.items()])  # noqa: E731
    old = {k: v for k, v in ck.items() if k != "layout"}
    old.update(format="vqa-vqvae/1", weights=pack(ck["weights"]), adam_m=pack(ck["adam_m"]), adam_v=pack(ck["adam_v"]))
    torch.save(old, str(tmp_path / "ckpt_v1.pt"))
    c = _model(cfg, B, dtype, R.init_params(cfg, 7), R.init_vq_state(cfg, 8))
    c.load(str(tmp_path / "ckpt_v1.pt"))
    torch.cuda.synchronize()
    assert torch.equal(c.store.flat.cpu(), ck["weights"]) and torch.equal(c.optimizer.m.cpu(), ck["adam_m"])
    a.train_step(xs[1])
    ra = {k: float(v) for k, v in a.train_step(xs[2]).items()}
    b = _model(cfg, B, dtype, R.init_params(cfg, 5), R.init_vq_state(cfg, 6))  # different start, then load
    b.load(path)
    b.train_step(xs[1])
    rb = {k: float(v) for k, v in b.train_step(xs[2]).items()}
    torch.cuda.synchronize()
    assert torch.equal(a.store.flat, b.store.flat)
    assert torch.equal(a.optimizer.m, b.optimizer.m) and torch.equal(a.optimizer.v, b.optimizer.v)
    for sa, sb in zip(a.get_vq_state(), b.get_vq_state()):
        for k in ("embeddings", "m_t", "N_t"):
            assert np.array_equal(sa[k], sb[k]), k
        assert sa["calls"] == sb["calls"] == 3
    # the last step's metrics (b's trackers saw two steps, a's three: compare the last step's contribution)
    assert a.loss_slots.cpu().equal(b.loss_slots.cpu())


def test_evaluate_keras_semantics(cuda):
    """VQVAE.evaluate (keras Model.evaluate, as src/callback/vae_monitor.py:69 calls it on the validation dataset):
    the model's trackers are reset, test_step (vqvae.py:148-172) runs on every batch — the codebook EMA included
    (VectorQuantizer.py:75 defaults training=True) — and the running means come back. Against the fp64 oracle's
    test_step sequence on the same two batches: loss keys rel 1e-5, codebook state after both batches (N_t on
    >= 99 % of codes, m_t / E relative L2 1e-4; a row on a near-tie may take the other code)."""
    c = CONFIGS["cfg1"]
    cfg, B = c["cfg"], c["B"]
    params, vq = R.init_params(cfg, 1), R.init_vq_state(cfg, 2)
    xs = [R.synthetic_batch(B, cfg.input_len, seed=70 + i) for i in range(3)]
    m = _model(cfg, B, "fp32", params, vq)
    m.train_step(xs[2])  # tracker state that evaluate must reset; the oracle starts from the state after it
    ref = R.RefVQVAE(cfg, params, vq, dtype=torch.float64)
    _sync_oracle(ref, m)
    logs = m.evaluate(xs[:2], return_dict=True)
    outs = [ref.test_step(x) for x in xs[:2]]
    for k in ("loss", "recon_loss", "vqvae_loss", "spectral_loss", "[0]level_loss", "[0]recon_loss", "[0]vq_loss",
              "[0]spectral_loss"):
        want = (outs[0][k] + outs[1][k]) / 2
        assert abs(logs[k] - want) <= 1e-5 * abs(want), (k, logs[k], want)
    st = m.get_vq_state()[0]
    assert st["calls"] == ref.vq[0]["calls"] == 3
    assert np.mean(np.isclose(st["N_t"], ref.vq[0]["N_t"].numpy(), rtol=1e-5, atol=0)) >= 0.99
    for k in ("m_t", "embeddings"):
        assert _l2(st[k], ref.vq[0][k].numpy()) < 1e-4, k
    # flattened in keras order: tracker names first (model.metrics order), then the other keys sorted
    flat = m.evaluate(np.concatenate(xs[:2]), batch_size=B)
    names = [t.name for t in m.metrics]
    order = [k for k in names if k in logs] + sorted(k for k in logs if k not in names)
    assert len(flat) == len(logs) and order[0] == "spectral_loss"
    assert m.evaluate(xs[:2], steps=1, return_dict=True).keys() == logs.keys()


def test_compile_after_capture_uses_new_optimizer(cuda):
    """Re-compiling after capture_train_step drops the captured step (it holds the old optimizer's m, v, step
    counter and learning rate): the next train_step runs with the new optimizer, eagerly, and equals a model that
    was compiled with it from the start."""
    from vqa_optim import Adam
    c = CONFIGS["cfg1"]
    cfg, B = c["cfg"], c["B"]
    params, vq = R.init_params(cfg, 1), R.init_vq_state(cfg, 2)
    xs = [R.synthetic_batch(B, cfg.input_len, seed=80 + i) for i in range(2)]
    a = _model(cfg, B, "fp32", params, vq)
    a.capture_train_step(xs[0], warmup=1)
    state = a.state_dict()
    a.compile(Adam(learning_rate=5e-4))
    assert a._graph is None
    a.train_step(xs[1])
    b = _model(cfg, B, "fp32", params, vq)
    b.compile(Adam(learning_rate=5e-4))
    b.store.flat.copy_(state["weights"].cuda())
    b.set_vq_state(state["vq"])
    b.train_step(xs[1])
    torch.cuda.synchronize()
    assert int(a.optimizer.iterations.item()) == 1
    assert torch.equal(a.store.flat, b.store.flat)


def test_repeated_step_bitwise(cuda):
    """Two models from the same state fed the same batches end bitwise identical (run-to-run determinism,
    SURVEY.md §5), eager and graph-replayed."""
    c = CONFIGS["cfg1"]
    cfg, B = c["cfg"], c["B"]
    params, vq = R.init_params(cfg, 1), R.init_vq_state(cfg, 2)
    xs = [R.synthetic_batch(B, cfg.input_len, seed=60 + i) for i in range(3)]
    runs = []
    for _ in range(2):
        m = _model(cfg, B, "bf16", params, vq)
        res = [m.train_step(x) for x in xs]
        torch.cuda.synchronize()
        runs.append((m.store.flat.clone(), [st["embeddings"] for st in m.get_vq_state()],
                     {k: float(v) for k, v in res[-1].items()}))
    assert torch.equal(runs[0][0], runs[1][0])
    for e0, e1 in zip(runs[0][1], runs[1][1]):
        assert np.array_equal(e0, e1)
    assert runs[0][2] == runs[1][2]


@pytest.mark.parametrize("name", ["cfg1", "tiny"])
def test_resblock_backward_teacher_forced(cuda, name):
    """Every residual block's backward (resnet.py:7-29) on the GPU vs fp64 autograd of the same block,
    fed the GPU's own saved input and upstream gradient, with ReLU masks taken from the GPU activations."""
    import torch.nn.functional as F
    import resnet
    c = CONFIGS[name]
    cfg, B = c["cfg"], c["B"]
    params, vq = R.init_params(cfg, 1), R.init_vq_state(cfg, 2)
    m = _model(cfg, B, "fp32", params, vq)
    log = []
    orig = resnet.ResnetConv1DBlock.backward

    def spy(self, dy):
        xs, h = self._saved
        fused = h is None
        if fused:  # fused block: relu(h) exactly as its backward recomputes it (vqa_resblock_fwd h_out)
            import vqa_lib as V
            h, y_ = torch.empty_like(xs), torch.empty_like(xs)
            V.resblock_fwd(xs, self.conv_a.w, self.conv_a.b, self.conv_b.w, self.conv_b.b, y_, self.dilation, h_out=h)
        rec = dict(blk=self, x=xs.double().cpu(), h=h.double().cpu(), dy=dy.double().cpu(), fused=fused)
        dx = orig(self, dy)
        rec["dx"] = dx.double().cpu()
        log.append(rec)
        return dx

    resnet.ResnetConv1DBlock.backward = spy
    try:
        m.train_step(R.synthetic_batch(B, cfg.input_len, seed=11))
    finally:
        resnet.ResnetConv1DBlock.backward = orig
    g = m.store.grads()
    assert len(log) == sum(1 for n in g if n.endswith("conv_a/kernel"))
    for rec in log:
        blk = rec["blk"]
        na, nb = blk.conv_a.name, blk.conv_b.name
        W = {k: torch.tensor(params[k], dtype=torch.float64, requires_grad=True)
             for k in (f"{na}/kernel", f"{na}/bias", f"{nb}/kernel", f"{nb}/bias")}
        xv = rec["x"].clone().requires_grad_(True)
        h = R.conv1d(xv * (rec["x"] > 0), W[f"{na}/kernel"], W[f"{na}/bias"], 1, blk.dilation)
        want_h = torch.relu(h) if rec["fused"] else h
        assert _l2(rec["h"].numpy(), want_h.detach().numpy()) < 1e-5, f"{na}: forward h"
        y = xv + R.conv1d(h * (rec["h"] > 0), W[f"{nb}/kernel"], W[f"{nb}/bias"], 1, 1)
        grads = torch.autograd.grad((y * rec["dy"]).sum(), [xv] + list(W.values()))
        assert _l2(rec["dx"].numpy(), grads[0].numpy()) < 1e-5, f"{na}: dx"
        for (k, _), gr in zip(W.items(), grads[1:]):
            assert _l2(g[k], gr.numpy()) < 1e-5, f"{k}"


def test_product_against_golden_micro(cuda, monkeypatch):
    """libvqa fp32 train steps vs the committed oracle fixture tests/golden/micro.npz (width 8, latent 4,
    K=64: the thin / generic kernel paths)."""
    import json
    import os
    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    z = np.load(os.path.join(gold, "micro.npz"))
    meta = json.load(open(os.path.join(gold, "micro.json")))
    cfg = R.RefConfig(**meta["config"])
    params = {k[5:]: z[k] for k in z.files if k.startswith("init/")}
    vq = [{"embeddings": z[f"vq_init{l}/embeddings"], "m_t": z[f"vq_init{l}/embeddings"],
           "N_t": np.ones(cfg.num_embeddings, np.float32), "calls": 0} for l in range(cfg.levels)]
    m = _model(cfg, meta["batch"], "fp32", params, vq)
    for s in range(meta["steps"]):
        vqlog = _capture_vq(monkeypatch)
        res = {k: float(v) for k, v in m.train_step(z[f"x{s}"]).items()}
        monkeypatch.undo()
        for rec in vqlog:  # the stored oracle indices, on every row clear of a tie by 1e-4 (fp32 vs fp64 z)
            l = rec["level"]
            clear = z[f"margin{s}_l{l}"] > 1e-4
            assert clear.mean() > 0.99
            got = rec["idx"].numpy()
            assert np.array_equal(got[clear], z[f"idx{s}_l{l}"][clear]), f"step {s} level {l}"
        want = {k: float(np.mean([meta["metrics"][i][k] for i in range(s + 1)])) for k in res}
        for k in res:
            tol = (1e-5 if s == 0 else 5e-5) if "usage" not in k and "entropy" not in k else 2e-2
            assert abs(res[k] - want[k]) <= tol * max(abs(want[k]), 1e-3), (s, k, res[k], want[k])
        g = m.store.grads()
        meds = [_rel(g[n[len(f"grad{s}/"):]], z[n]) for n in z.files if n.startswith(f"grad{s}/")]
        assert np.median(meds) < 5e-4
    w = m.get_weights()
    for n in params:
        assert _l2(w[n], z[f"final/{n}"]) < 1e-3, n


def test_product_against_golden_cfg1_scalars(cuda):
    import json
    import os
    meta = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cfg1.json")))
    cfg = R.RefConfig(**meta["config"])
    m = _model(cfg, meta["batch"], "fp32", R.init_params(cfg, 1), R.init_vq_state(cfg, 2))
    res = {k: float(v) for k, v in m.train_step(R.synthetic_batch(meta["batch"], cfg.input_len,
                                                                   seed=meta["x_seeds"][0])).items()}
    for k in ("loss", "recon_loss", "vqvae_loss", "spectral_loss", "[0]batch_codebook_usage"):
        assert abs(res[k] - meta["metrics"][0][k]) <= 1e-5 * max(abs(meta["metrics"][0][k]), 1e-3), k
    g = m.store.grads()
    rel = [abs(np.linalg.norm(g[n]) - v) / v for n, v in meta["grad_norms"][0].items()]
    assert np.median(rel) < 2e-4 and max(rel) < 5e-3  # gradient norms: ReLU-kink sensitive (see module doc)


def _spy_convs(monkeypatch):
    """Record every Conv1D / Conv1DTranspose call of a real step (inputs and outputs copied to host)."""
    import vqa_layers as L
    log = []

    def host(t):
        return None if t is None else t.detach().double().cpu()

    def wrap(cls, meth, kind):
        orig = getattr(cls, meth)

        def f(self, *args, **kw):
            out = orig(self, *args, **kw)
            torch.cuda.synchronize()
            rec = {"kind": kind, "layer": self, "args": [host(a) if isinstance(a, torch.Tensor) else a for a in args],
                   "kw": {k: host(v) if isinstance(v, torch.Tensor) else v for k, v in kw.items()},
                   "out": host(out)}
            log.append(rec)  # weight gradients are read after the step (their reduction is deferred)
            return out
        monkeypatch.setattr(cls, meth, f)

    for cls, tag in ((L.Conv1D, "conv"), (L.Conv1DTranspose, "convT")):
        for meth in ("forward", "backward_data", "backward_weight", "backward_data_weight"):
            if hasattr(cls, meth):
                wrap(cls, meth, (tag, meth))
    return log


@pytest.mark.parametrize("name,dtype", [("cfg1", "fp32"), ("tiny", "fp32"), ("cfg2_short", "fp32")])
def test_every_conv_call_teacher_forced(cuda, monkeypatch, name, dtype):
    """Every conv kernel call of a real train step (forward, data-gradient, weight-gradient; fused ReLU,
    residual and ReLU' masks) against fp64 autograd of the oracle's TF-semantics conv on the SAME
    inputs and masks the GPU used. No branch can flip, so the bound is strict (relative L2 1e-5)."""
    c = CONFIGS[name]
    cfg, B = c["cfg"], c["B"]
    params, vq = R.init_params(cfg, 1), R.init_vq_state(cfg, 2)
    m = _model(cfg, B, dtype, params, vq)
    log = _spy_convs(monkeypatch)
    m.train_step(R.synthetic_batch(B, cfg.input_len, seed=11))
    monkeypatch.undo()
    assert log
    g = m.store.grads()
    for rec in log:
        if rec["kind"][1] in ("backward_weight", "backward_data_weight"):
            rec["dw"] = torch.from_numpy(g[f"{rec['layer'].name}/kernel"]).double()
            rec["db"] = torch.from_numpy(g[f"{rec['layer'].name}/bias"]).double()
    worst = 0.0
    for rec in log:
        tag, meth = rec["kind"]
        lay = rec["layer"]
        W = torch.tensor(params[f"{lay.name}/kernel"], dtype=torch.float64, requires_grad=True)
        b = torch.tensor(params[f"{lay.name}/bias"], dtype=torch.float64, requires_grad=True)
        if tag == "conv":
            f = lambda x, W, b: R.conv1d(x, W, b, lay.s, lay.d)  # noqa: E731
        else:
            f = lambda x, W, b: R.conv1d_transpose(x, W, b, lay.s)  # noqa: E731
        kw = rec["kw"]
        if meth == "forward":
            x = rec["args"][0]
            if kw.get("pre_relu"):
                x = x * (x > 0)
            want = f(x, W, b)
            if kw.get("residual") is not None:
                want = kw["residual"] + want
            err = _l2(rec["out"].numpy(), want.detach().numpy())
        elif meth == "backward_data":
            dy = rec["args"][0]
            T_in = rec["args"][1] if tag == "conv" else dy.shape[1] // lay.s
            xv = torch.zeros(dy.shape[0], T_in, lay.cin, dtype=torch.float64, requires_grad=True)
            (gx,) = torch.autograd.grad((f(xv, W, b) * dy).sum(), xv)
            if kw.get("mask") is not None:
                gx = gx * (kw["mask"] > 0)
            if kw.get("residual") is not None:
                gx = kw["residual"] + gx
            err = _l2(rec["out"].numpy(), gx.numpy())
        elif meth == "backward_data_weight":  # fused: dx (ReLU' mask = the conv input) and dW, db
            dy, x0 = rec["args"][0], rec["args"][1]
            xv = x0.clone().requires_grad_(True)
            x = xv * (xv > 0) if kw.get("pre_relu") else xv
            gx, gW, gb = torch.autograd.grad((f(x, W, b) * dy).sum(), (xv, W, b))
            if kw.get("residual") is not None:
                gx = kw["residual"] + gx
            err = max(_l2(rec["out"].numpy(), gx.numpy()), _l2(rec["dw"].numpy(), gW.numpy()),
                      _l2(rec["db"].numpy(), gb.numpy()))
        else:
            x, dy = rec["args"][0], rec["args"][1]
            if kw.get("pre_relu"):
                x = x * (x > 0)
            gW, gb = torch.autograd.grad((f(x, W, b) * dy).sum(), (W, b))
            err = max(_l2(rec["dw"].numpy(), gW.numpy()), _l2(rec["db"].numpy(), gb.numpy()))
        worst = max(worst, err)
        assert err < 1e-5, f"{lay.name} {meth}: relative L2 {err:.3e}"
    print(f"{len(log)} conv calls checked, worst relative L2 {worst:.2e}")


REF_METRIC_NAMES = lambda L: (["total_loss", "reconstruction_loss", "vq_loss", "spectral_loss"] +  # noqa: E731
                              [f"[{l}]{k}" for k in ("level_loss", "recon_loss", "vq_loss", "spectral_loss")
                               for l in range(L)])


def test_keras_metric_trackers_and_monitor_reset(cuda):
    """vqvae.py:93-104 `metrics` are keras Mean trackers (name / result / reset_state) in the reference order,
    backed by the device accumulator the step updates; the monitor's loop (src/callback/vae_monitor.py:64-65,
    71) resets them; the VQ usage trackers (VectorQuantizer.metrics) are wired to the step and, not being
    in `model.metrics`, keep accumulating (keras semantics of the reference)."""
    c = CONFIGS["tiny"]
    cfg, B = c["cfg"], c["B"]
    m = _model(cfg, B, "fp32", R.init_params(cfg, 1), R.init_vq_state(cfg, 2))
    assert [t.name for t in m.metrics] == REF_METRIC_NAMES(cfg.levels)
    res = {k: float(v) for k, v in m.train_step(R.synthetic_batch(B, cfg.input_len, seed=3)).items()}
    assert float(m.metrics[0].result()) == res["loss"]
    assert float(m.metrics[4].result()) == res["[0]level_loss"]
    vq_usage = {t.name: float(t.result()) for vq in m.vqs for t in vq.metrics}
    for k, v in vq_usage.items():
        assert v == res[k] and v > 0, k
    for t in m.metrics:                       # vae_monitor.py:64-65
        t.reset_state()
    logged = {f"[val]{t.name}": float(t.result()) for t in m.metrics}  # vae_monitor.py:70-72
    assert all(v == 0.0 for v in logged.values())
    assert {t.name: float(t.result()) for vq in m.vqs for t in vq.metrics} == vq_usage
    res2 = {k: float(v) for k, v in m.test_step(R.synthetic_batch(B, cfg.input_len, seed=4)).items()}
    assert float(m.metrics[0].result()) == res2["loss"]  # one value since the reset


def test_get_vqvae_single_level_model(cuda):
    """vqvae.py:15-21 get_vqvae(input_shape, encoder, decoder, vq, level): x -> encoder -> vq -> decoder on a
    fixed input shape; against the oracle's level forward with the same weights."""
    from encdec import Decoder, Encoder
    from vqvae import get_vqvae
    from VectorQuantizer import VectorQuantizer
    cfg = R.RefConfig(input_len=2048, levels=1, latent_dim=8, down_depth=[2], strides=[2], num_embeddings=64,
                      residual_width=32, residual_depth=2, dilation_factor=3)
    enc = Encoder(cfg.latent_dim, cfg.residual_width, cfg.residual_depth, 1, cfg.down_depth, cfg.strides,
                  cfg.dilation_factor)
    dec = Decoder(1, cfg.latent_dim, cfg.residual_width, cfg.residual_depth, 1, cfg.down_depth, cfg.strides,
                  cfg.dilation_factor)
    vq = VectorQuantizer(cfg.num_embeddings, cfg.latent_dim, device=cuda)
    model = get_vqvae((cfg.input_len, 1), enc, dec, vq, level=0)
    assert model.name == "vq_vae_0" and len(model.trainable_variables) == len(R.param_specs(cfg))
    params = model.store.values()
    vqs = [{"embeddings": vq.embeddings.cpu().numpy(), "m_t": vq.m_t.cpu().numpy(), "N_t": vq.N_t.cpu().numpy()}]
    ref = R.RefVQVAE(cfg, params, vqs, dtype=torch.float64)
    x = R.synthetic_batch(2, cfg.input_len, seed=8)
    y = model(x, training=False)
    want = ref.level_forward(torch.as_tensor(x, dtype=torch.float64), 0, training=False)["recon"]
    assert tuple(y.shape) == (2, cfg.input_len, 1)
    assert _rel(y.cpu().numpy(), want.detach().numpy()) < 1e-4
    assert len(model.losses) == 1 and float(model.losses[0]) > 0
    with pytest.raises(ValueError):
        model(R.synthetic_batch(2, 1024, seed=8))


def test_update_metrics_and_multispectral_loss_api(cuda):
    """vqvae.py:262-304 update_metrics on given per-level losses (trackers = running means of the sums / the
    per-level values, the reference's key set) and vqvae.py:309-326 _multispectral_loss (the product's
    spectral-loss kernel through the reference's method name) vs the oracle's loss on the same reconstruction."""
    from oracle import vqvae_ref as R
    from vqvae import VQVAE
    m = VQVAE((4096, 1), 2, 64, [3, 2], [2, 2], num_embeddings=64, residual_width=32, residual_depth=2,
              dilation_factor=3, dtype="fp32", device="cuda")
    for t in m.metrics:
        t.reset_state()
    out1 = m.update_metrics([1.0, 2.0], [0.5, 0.25], [0.125, 0.0625], [0.375, 1.6875])
    out2 = m.update_metrics([3.0, 4.0], [0.5, 0.75], [0.125, 0.1875], [2.375, 3.0625])
    assert float(out2["loss"]) == 5.0 and float(out2["recon_loss"]) == 1.0
    assert abs(float(out2["vqvae_loss"]) - 0.25) < 1e-7 and abs(float(out2["spectral_loss"]) - 3.75) < 1e-6
    assert float(m.level_loss_trackers[1].result()) == 3.0 and float(m.recon_loss_trackers[0].result()) == 0.5
    per_level = {t.name for ts in (m.level_loss_trackers, m.recon_loss_trackers, m.vq_loss_trackers,
                                   m.spectral_loss_trackers) for t in ts}
    vq_names = {t.name for vq in m.vqs for t in vq.metrics}
    assert set(out1) == {"loss", "recon_loss", "vqvae_loss", "spectral_loss"} | per_level | vq_names
    x = R.synthetic_batch(2, 4096, seed=5)
    r = x + 0.05 * np.random.default_rng(1).standard_normal(x.shape).astype(np.float32)
    got = float(m._multispectral_loss(torch.from_numpy(x).cuda(), torch.from_numpy(r).cuda()))
    ref = float(R.multispectral_loss(torch.from_numpy(x).double(), torch.from_numpy(r).double()).mean())
    assert abs(got - ref) <= 1e-5 * abs(ref)
