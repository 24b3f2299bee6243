"""The prior oracle (oracle/prior_ref.py) against the reference's own consistency check and known answers (CPU)."""
import math

import numpy as np
import pytest
import torch

from oracle import prior_ref as P


TINY = P.PriorConfig(bins=17, ctx=16, width=16, depth=3, heads=2, blocks=4, attn_stacks=1)


def _params(cfg, seed=3):
    return P.to_torch(P.init_params(cfg, seed))


def test_keras_fans_and_init_limits():
    assert P.keras_fans((32, 2, 16)) == (64, 512)       # EinsumDense kernel: receptive field = 32
    assert P.keras_fans((3, 128, 96)) == (384, 288)     # Conv1D kernel
    assert P.keras_fans((128, 2048)) == (128, 2048)     # Dense kernel
    vals = P.init_params(TINY, 1)
    lim = math.sqrt(6.0 / (3 * 16 + 3 * 12))
    w = vals["prior/layer0/qkv/kernel"]
    assert w.shape == (3, 16, 12) and np.abs(w).max() <= lim


def test_look_ahead_mask():
    m = P.look_ahead_mask(3, 3)
    assert torch.equal(m, torch.tensor([[1., 0, 0], [1, 1, 0], [1, 1, 1]], dtype=torch.float64))


@pytest.mark.parametrize("attn", [0, 1, 2])
def test_prefix_calls_equal_full_call(attn):
    """factorized_attention.py:446-462: every prefix call of the attention layer equals the full call at those
    positions (the reference asserts max |diff| <= 1e-6)."""
    cfg = P.PriorConfig(bins=17, ctx=16, width=16, depth=1, heads=2, blocks=4)
    p = _params(cfg)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 16, 16, generator=g, dtype=torch.float64)
    pre = "prior/layer0"
    full = P.res_attn_block(p, pre, x, attn, cfg.block_len)
    for i in range(16):
        part = P.res_attn_block(p, pre, x[:, :i + 1], attn, cfg.block_len)
        assert (part - full[:, :i + 1]).abs().max() <= 1e-12


def test_model_prefix_equals_full_and_causal():
    p = _params(TINY)
    tok = torch.randint(0, TINY.bins, (2, 16), generator=torch.Generator().manual_seed(1))
    full = P.model_forward(p, TINY, tok)
    for i in (0, 3, 4, 9, 15):
        part = P.model_forward(p, TINY, tok[:, :i + 1])
        assert (part - full[:, :i + 1]).abs().max() <= 1e-12
    tok2 = tok.clone()
    tok2[:, 10:] = (tok2[:, 10:] + 1) % TINY.bins  # future tokens do not change earlier logits
    assert (P.model_forward(p, TINY, tok2)[:, :10] - full[:, :10]).abs().max() == 0


def test_prev_row_first_block_is_value_bias():
    """prev_row_attn pads a zero block: block 0's queries see keys = key bias, values = value bias, so the
    MHA output there is out_dense(value bias)."""
    cfg = P.PriorConfig(bins=5, ctx=8, width=16, depth=1, heads=2, blocks=2)
    p = _params(cfg)
    p["prior/layer0/mha/value/bias"] = torch.randn(2, 2, dtype=torch.float64)
    p["prior/layer0/mha/key/bias"] = torch.randn(2, 2, dtype=torch.float64)
    q, k, v = (torch.randn(1, 8, 4, dtype=torch.float64) for _ in range(3))
    o = P.prev_row_attn(p, "prior/layer0/mha", q, k, v, 4)
    want = torch.einsum("cd,cde->e", p["prior/layer0/mha/value/bias"], p["prior/layer0/mha/out/kernel"]) + \
        p["prior/layer0/mha/out/bias"]
    assert (o[0, :4] - want).abs().max() < 1e-12


def test_col_attention_known_answer():
    """One head, identity projections: position j of block b averages (softmax-weights) positions j of blocks <= b."""
    cfg = P.PriorConfig(bins=5, ctx=6, width=8, depth=1, heads=1, blocks=3)
    p = _params(cfg)
    pre = "prior/layer0/mha"
    w = cfg.attn_width  # 2
    for n in ("query", "key", "value"):
        p[f"{pre}/{n}/kernel"] = torch.eye(w, dtype=torch.float64).reshape(w, 1, w)
        p[f"{pre}/{n}/bias"] = torch.zeros(1, w, dtype=torch.float64)
    p[f"{pre}/out/kernel"] = torch.eye(w, dtype=torch.float64).reshape(1, w, w)
    p[f"{pre}/out/bias"] = torch.zeros(w, dtype=torch.float64)
    q = torch.zeros(1, 6, w, dtype=torch.float64)  # zero queries: uniform weights over the visible keys
    v = torch.arange(12, dtype=torch.float64).reshape(1, 6, w)
    o = P.col_attn(p, pre, q, q, v, 2)
    # block len 2: positions 0,2,4 form column 0; 1,3,5 column 1
    assert torch.allclose(o[0, 4], (v[0, 0] + v[0, 2] + v[0, 4]) / 3)
    assert torch.allclose(o[0, 3], (v[0, 1] + v[0, 3]) / 2)
    assert torch.allclose(o[0, 1], v[0, 1])


def test_ce_loss_accuracy_known_answer():
    logits = torch.tensor([[[0.0, math.log(3.0)], [2.0, 2.0]]], dtype=torch.float64)
    tgt = torch.tensor([[1, 1]])
    assert abs(float(P.ce_loss(tgt, logits)) - (math.log(4 / 3) + math.log(2)) / 2) < 1e-12
    assert float(P.accuracy(tgt, logits)) == 0.5  # the tie resolves to index 0 (tf.argmax)


def test_train_step_teacher_forcing_mix():
    p = _params(TINY)
    codes = torch.randint(0, TINY.bins - 1, (2, 16), generator=torch.Generator().manual_seed(2))
    none = torch.zeros(2, 16, dtype=torch.bool)
    loss, acc, grads, bi = P.train_step_grads(p, TINY, codes, none)
    assert torch.equal(bi, P.shift_right(codes, TINY.bins - 1))
    assert set(grads) == set(p) and all(torch.isfinite(g).all() for g in grads.values())
    allm = torch.ones(2, 16, dtype=torch.bool)
    _, _, _, bi2 = P.train_step_grads(p, TINY, codes, allm)
    assert (bi2[:, 0] == TINY.bins - 1).all()
    assert 0 < loss < 10 and 0 <= acc <= 1


def test_gumbel_uniform_range_and_determinism():
    u = P.gumbel_uniform(7, 1, 5, np.arange(4096))
    assert u.min() > 0 and u.max() < 1 and abs(float(u.mean()) - 0.5) < 0.02
    assert np.array_equal(u, P.gumbel_uniform(7, 1, 5, np.arange(4096)))
    assert not np.array_equal(u, P.gumbel_uniform(7, 2, 5, np.arange(4096)))


def test_sampler_reference_recompute_small():
    p = _params(TINY)
    out, margins = P.sample_full_recompute(p, TINY, 2, 6, seed=11)
    assert out.shape == (2, 7) and (out[:, 0] == TINY.bins - 1).all()
    assert ((out >= 0) & (out < TINY.bins)).all()
