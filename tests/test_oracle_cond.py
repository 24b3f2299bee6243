"""Host tests of the conditioner (no GPU): the oracle's LayerNorm / Embedding / cyclic-dilation semantics
against hand-derived known answers, and the product ConditionerNet's parameter registration (names, shapes,
keras initialisers) against the oracle's naming (src/conditioner/conditioners.py:42-72)."""
import numpy as np
import torch

from conditioners import ConditionerNet
from oracle import conditioner_ref as CR
from vqa_layers import ParamStore


def test_layer_norm_known_answer():
    x = torch.tensor([[1.0, 2.0, 3.0, 4.0]], dtype=torch.float64)
    g = torch.tensor([1.0, 2.0, 1.0, 1.0], dtype=torch.float64)
    b = torch.tensor([0.0, 0.0, 1.0, 0.0], dtype=torch.float64)
    y = CR.layer_norm(x, g, b, eps=1e-6)
    # mean 2.5, var 1.25
    s = 1.0 / np.sqrt(1.25 + 1e-6)
    want = np.array([-1.5 * s, -0.5 * s * 2, 0.5 * s + 1.0, 1.5 * s])
    assert np.allclose(y.numpy()[0], want, rtol=0, atol=1e-12)


def test_cyclic_dilations():
    """resnet.py:44-55 with the prior's x_cond_kwargs (dilation_factor 3, dilation_cycle 4, depth 8)."""
    assert CR.dilations(8, 3, False, 4) == [1, 3, 9, 27, 1, 3, 9, 27]
    assert CR.dilations(8, 3, True, 4) == [27, 9, 3, 1, 27, 9, 3, 1]
    assert CR.dilations(4, 3, False, None) == [1, 3, 9, 27]


def test_conditioner_parameters_and_forward_shapes():
    net = ConditionerNet((16,), bins=10, embed_width=128, residual_width=32, residual_depth=8, down_depth=3,
                         stride=2, dilation_factor=3, dilation_cycle=4)
    store = ParamStore()
    assert net.build(store, "cond", 128, torch.float32) == 128
    names = dict((n, s) for n, s, _ in store.specs)
    assert names["cond/embedding/embeddings"] == (10, 128)
    assert names["cond/block/pre/kernel"] == (3, 128, 32)
    assert names["cond/block/up2/kernel"] == (4, 128, 32)   # Conv1DTranspose (K, C_out, C_in): 32 -> 128
    assert names["cond/layer_norm/gamma"] == (128,)
    # 8 blocks per residual stack, cyclic dilations 1, 3, 9, 27
    assert [b.dilation for b in net.block.res[0].blocks] == [1, 3, 9, 27, 1, 3, 9, 27]
    vals = store.init_values(1)
    assert np.abs(vals["cond/embedding/embeddings"]).max() <= 0.05
    assert (vals["cond/layer_norm/gamma"] == 1).all() and (vals["cond/layer_norm/beta"] == 0).all()
    # the oracle consumes the same names: output length L * stride^down_depth
    p = {k: torch.tensor(v, dtype=torch.float64) for k, v in vals.items()}
    y = CR.conditioner_forward(p, torch.randint(0, 10, (2, 16)), "cond", 3, 2, 8, 3, False, 4)
    assert tuple(y.shape) == (2, 128, 128) and net.out_len() == 128
    assert torch.allclose(y.mean(-1), torch.zeros(2, 128, dtype=torch.float64), atol=1e-9)
