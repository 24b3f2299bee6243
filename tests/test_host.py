"""Host-side logic, no GPU: the product's layer structure / parameter registration / init vs the oracle,
the DP bucket layout, dilation schedules, and the loud failure modes of the C-ABI binding."""
import numpy as np
import pytest
import torch

import vqa_dp
import vqa_lib as V
from encdec import Decoder, Encoder
from oracle import vqvae_ref as R
from resnet import DilatedResnet1D
from vqa_layers import ParamStore

CFG2 = R.RefConfig(input_len=65536, levels=3, latent_dim=64, down_depth=[3, 2, 2], strides=[2, 2, 2],
                   num_embeddings=2048, residual_width=32, residual_depth=4, dilation_factor=3)
CFG1 = R.RefConfig(input_len=4096, levels=1, latent_dim=64, down_depth=[3], strides=[2], num_embeddings=256,
                   residual_width=32, residual_depth=4, dilation_factor=3)
TINY = R.RefConfig(input_len=2048, levels=2, latent_dim=8, down_depth=[2, 1], strides=[2, 2], num_embeddings=1024,
                   residual_width=32, residual_depth=2, dilation_factor=3)


def _product_store(cfg):
    store = ParamStore()
    for l in range(cfg.levels):
        enc = Encoder(cfg.latent_dim, cfg.residual_width, cfg.residual_depth, l + 1, cfg.down_depth[:l + 1],
                      cfg.strides[:l + 1], cfg.dilation_factor)
        dec = Decoder(1, cfg.latent_dim, cfg.residual_width, cfg.residual_depth, l + 1, cfg.down_depth[:l + 1],
                      cfg.strides[:l + 1], cfg.dilation_factor)
        assert enc.build(store, f"enc{l}", 1, torch.bfloat16) == cfg.latent_dim
        assert dec.build(store, f"dec{l}", cfg.latent_dim, torch.bfloat16) == 1
    return store


@pytest.mark.parametrize("cfg", [CFG2, TINY])
def test_parameter_structure_matches_oracle(cfg):
    store = _product_store(cfg)
    assert [(n, s) for n, s, _ in store.specs] == R.param_specs(cfg)


def test_cfg2_parameter_count():
    """968,835 trainable parameters in 570 tensors at cfg2."""
    store = _product_store(CFG2)
    assert store.count == 968835 and len(store.specs) == 570 and store.size >= store.count
    assert all(off % 4 == 0 for off, _ in store.offsets.values())  # 16-byte aligned tensors


def test_init_matches_oracle_bitwise():
    store = _product_store(TINY)
    want = R.init_params(TINY, 1)
    got = store.init_values(1)
    assert got.keys() == want.keys()
    for n in want:
        assert np.array_equal(got[n], want[n]), n


@pytest.mark.parametrize("depth,f,rev,cycle,want", [(4, 3, False, None, [1, 3, 9, 27]), (4, 3, True, None, [27, 9, 3, 1]),
                                                    (8, 3, False, 4, [1, 3, 9, 27, 1, 3, 9, 27]), (3, 1, False, None, [1, 1, 1])])
def test_dilation_schedule(depth, f, rev, cycle, want):
    """resnet.py:44-55."""
    assert DilatedResnet1D(32, depth, f, rev, cycle).dilations == want


def test_bucket_layout_cfg2():
    stats = [2 * 2048 * 64 + 2048] * 3
    lay = vqa_dp.bucket_layout(968835, stats, 3)
    P0, P1 = lay["grads"]
    assert P0 == 0 and P1 >= 968835 and P1 % 64 == 0
    prev = P1
    for a, b in lay["stats"]:
        assert a == prev and b - a == stats[0]
        prev = b
    assert lay["losses"] == (prev, prev + 9) and lay["total"] == prev + 9
    mb = lay["total"] * 4 / 1e6
    # 7.0 MB per step on the wire at cfg2: 3.9 MB grads + 3 x (m_sum 0.5 MB + n_sum + reset rows 0.5 MB)
    assert 6.5 < mb < 7.5, mb
    sl = vqa_dp.vq_stats_slices(2048, 64)
    assert sl["m_sumT"] == (0, 131072) and sl["n_sum"] == (131072, 133120) and sl["RT"][1] == stats[0]


@pytest.mark.parametrize("cfg", [CFG2, TINY, CFG1])
def test_level_regions_partition_the_bucket(cfg):
    """The overlapped exchange (vqa_dp.level_regions): per level its layers' gradient range and its VQ statistics;
    the gradient ranges tile [0, P) in level order and contain every parameter of that level, so the per-level
    sums plus the losses cover exactly the one-bucket exchange."""
    store = _product_store(cfg)
    K, D = cfg.num_embeddings, cfg.latent_dim
    lay = vqa_dp.bucket_layout(store.size, [2 * K * D + K] * cfg.levels, cfg.levels)
    ranges = vqa_dp.level_param_ranges(store.offsets, cfg.levels)
    regs = vqa_dp.level_regions(lay, ranges)
    cover = np.zeros(lay["total"], np.int32)
    for l, (g, st) in enumerate(regs):
        for a, b in (g, st):
            cover[a:b] += 1
        assert st == lay["stats"][l]
        for n, (o, sh) in store.offsets.items():
            if n.startswith((f"enc{l}/", f"dec{l}/")):
                assert g[0] <= o and o + int(np.prod(sh)) <= g[1], n
    a, b = lay["losses"]
    cover[a:b] += 1
    assert (cover == 1).all()
    assert regs[0][0][0] == 0 and regs[-1][0][1] == lay["grads"][1]
    if cfg.levels > 1:  # a level range that starts inside the previous level's is refused
        with pytest.raises(ValueError):
            vqa_dp.level_regions(lay, [ranges[0]] + [(ranges[0][0], r[1]) for r in ranges[1:]])


def test_single_rank_dp_helpers():
    assert vqa_dp.world_size() == 1 and vqa_dp.rank() == 0
    assert vqa_dp.global_row_range(1000) == (0, 1000)
    b = torch.ones(10)
    assert vqa_dp.exchange(b) == 1 and float(b.sum()) == 10


def test_binding_rejects_host_tensors():
    with pytest.raises(V.VQAError, match="device tensors"):
        V.ptr(torch.zeros(4))


def test_binding_fails_loudly_without_library(monkeypatch):
    monkeypatch.setattr(V, "LIB_PATH", "/nonexistent/libvqa.so")
    monkeypatch.setattr(V, "_lib", None)
    with pytest.raises(ImportError, match="no CPU fallback"):
        V.lib()


def test_keras_mean_trackers_monitor_loop():
    """vqa_metrics.Mean / SlotMean have the keras tracker surface the reference's monitor uses
    (src/callback/vae_monitor.py:64-65 reset loop, :70-72 name / result)."""
    from vqa_metrics import Mean, SlotMean
    acc = torch.zeros(3, 2)
    ts = [SlotMean(f"m{i}", acc, i) for i in range(3)]
    for i, t in enumerate(ts):
        t.update_state(torch.tensor(float(i + 1)))
        t.update_state(torch.tensor(float(3 * (i + 1))))
    assert [float(t.result()) for t in ts] == [2.0, 4.0, 6.0]
    for t in ts[:2]:
        t.reset_state()
    assert [float(t.result()) for t in ts] == [0.0, 0.0, 6.0] and float(acc[2, 1]) == 2.0
    m = Mean("x", "cpu")
    m.update_state(torch.tensor(5.0))
    m.reset_states()
    assert float(m.result()) == 0.0 and m.name == "x"


def test_splitsongs_and_tile():
    """data_utils.py:65-91 splitsongs (hand-derived: T=100, window 0.2 -> chunk 20, overlap 0.5 -> hop 10, starts
    0..80 -> 9 chunks) and VectorQuantizer._tile (:191-199: ceil(K/N) repeats when N < K)."""
    import numpy as np
    import torch
    from data_utils import splitsongs
    from VectorQuantizer import VectorQuantizer
    x = np.arange(100, dtype=np.float32)
    xs, ys = splitsongs(x, 3, window=0.2, overlap=0.5)
    assert xs.shape == (9, 20) and ys.tolist() == [3] * 9
    assert xs[1, 0] == 10 and xs[-1, -1] == 99
    xs2, _ = splitsongs(np.stack([x, -x]), 1, window=0.2, overlap=0.5)
    assert xs2.shape == (9, 2, 20) and xs2[2, 1, 0] == -20
    xs3, _ = splitsongs(np.arange(95, dtype=np.float32), 0, window=0.2, overlap=0.0)  # chunk 19, hop 19: 5 chunks
    assert xs3.shape == (5, 19)
    from types import SimpleNamespace
    vq = SimpleNamespace(num_embeddings=8)  # _tile reads only K (the real layer allocates device state)
    t = VectorQuantizer._tile(vq, torch.arange(12.).reshape(3, 4))
    assert t.shape == (9, 4) and torch.equal(t[3:6], t[:3])
    assert VectorQuantizer._tile(vq, torch.zeros(10, 4)).shape == (10, 4)


def test_lr_schedules_host_values():
    """src/transformer/multi_head_attention.py:82-101 CustomSchedule in TF float32 arithmetic, and keras
    ExponentialDecay; the device kernel's constants come from the same host rounding."""
    from schedules import CustomSchedule, ExponentialDecay
    s = CustomSchedule(128, warmup_steps=4000)
    f32 = np.float32
    for step in (1, 10, 3999, 4000, 4001, 100000):
        want = f32(f32(1) / np.sqrt(f32(128))) * min(f32(1) / np.sqrt(f32(step)), f32(f32(step) * f32(4000 ** -1.5)))
        assert s(step) == float(f32(want)), step
    assert s(0) == 0.0
    peak = max(s(t) for t in (3999, 4000, 4001))
    assert abs(peak - 128 ** -0.5 * 4000 ** -0.5) < 1e-9
    kind, p = s.device_spec()
    assert kind == 1 and p[0] == float(f32(1) / np.sqrt(f32(128)))
    e = ExponentialDecay(0.1, 10, 0.5, staircase=True)
    assert e(9) == float(f32(0.1)) and e(10) == float(f32(0.05)) and e(25) == float(f32(0.025))
    assert abs(ExponentialDecay(0.1, 10, 0.5)(5) - 0.1 * 0.5 ** 0.5) < 1e-8


def test_adam_rejects_host_callables():
    from vqa_optim import Adam
    with pytest.raises(TypeError):
        Adam(learning_rate=lambda step: 1e-3)


def test_checkpoint_layouts_v1_packed_v1_aligned_v2():
    """Checkpoint format /2 records each tensor's [offset, *shape]; a /1 file is read in the layout its length
    identifies — the 16-byte-aligned one or the packed one of the first releases — and copied by name into the
    aligned layout; anything else is rejected with a clear error."""
    from vqa_layers import CKPT_VERSION, checkpoint_layout
    st = ParamStore()
    for n, s in (("a/bias", (1,)), ("b/kernel", (3, 1, 2)), ("c/bias", (5,)), ("d/kernel", (2, 2))):
        st.add(n, s, "zeros")
    assert st.count == 16 and st.size == 24  # offsets 0, 4, 12, 20
    vals = {n: np.arange(int(np.prod(s)), dtype=np.float32).reshape(s) + 10 * i
            for i, (n, s, _) in enumerate(st.specs)}
    aligned = torch.zeros(st.size)
    for n, (o, s) in st.offsets.items():
        aligned[o:o + int(np.prod(s))] = torch.from_numpy(vals[n].reshape(-1))
    packed = torch.cat([torch.from_numpy(vals[n].reshape(-1)) for n, _, _ in st.specs])
    names = [n for n, _, _ in st.specs]
    for flat in (aligned, packed):
        ck = {"format": "vqa-vqvae/1", "param_names": names, "weights": flat}
        lay = checkpoint_layout(ck, st, "vqvae", "x.pt")
        assert torch.equal(st.from_layout(flat, lay, "x.pt"), aligned)
    ck2 = {"format": f"vqa-vqvae/{CKPT_VERSION}", "layout": st.layout_record(), "weights": aligned}
    assert torch.equal(st.from_layout(aligned, checkpoint_layout(ck2, st, "vqvae", "y.pt"), "y.pt"), aligned)
    with pytest.raises(ValueError, match="fits neither"):
        checkpoint_layout({"format": "vqa-vqvae/1", "param_names": names, "weights": torch.zeros(17)}, st, "vqvae", "z")
    with pytest.raises(ValueError, match="differs"):
        checkpoint_layout({"format": "vqa-vqvae/1", "param_names": names[::-1], "weights": packed}, st, "vqvae", "z")
    with pytest.raises(ValueError, match="not a vqa-prior"):
        checkpoint_layout(ck2, st, "prior", "z")
    bad = st.layout_record()
    bad["c/bias"] = [12, 4]
    with pytest.raises(ValueError, match="shape"):
        st.from_layout(aligned, bad, "w")
