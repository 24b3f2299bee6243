"""CPU restatement (torch, fp64 by default) of the reference ConditionerNet. TEST INFRASTRUCTURE ONLY.

src/conditioner/conditioners.py:62-72  keras.Sequential([
    layers.Embedding(bins, width),                                      -> table[idx]
    DecoderConvBlock(width, residual_width, residual_depth, stride, dilation_factor, reverse_dilation,
                     down_depth, dilation_cycle),                       -> encdec.py:44-71 + resnet.py:7-59
    layers.LayerNormalization(axis=-1, epsilon=1e-6)])                  -> tf.nn.moments + batch_normalization
Parameter names follow the product's ParamStore layout (conditioners.py: prefix/embedding/embeddings,
prefix/block/{pre, res{i}/rb{j}/conv_{a,b}, up{i}}, prefix/layer_norm/{gamma, beta}).
Parity unpinned (TensorFlow is not importable here; the reference holds no fixtures for this layer): pinned
by the KATs of its parts (tests/test_oracle_kat.py: SAME padding, Conv1DTranspose alignment) and by
tests/test_oracle_cond.py (LayerNorm / Embedding known answers, cyclic dilation schedule).
"""
from typing import Dict

import torch
import torch.nn.functional as F

from oracle.vqvae_ref import conv1d, conv1d_transpose


def dilations(depth, factor, reverse, cycle):
    """resnet.py:44-55."""
    d = [factor ** (i if cycle is None else i % cycle) for i in range(depth)]
    return d[::-1] if reverse else d


def layer_norm(x, gamma, beta, eps=1e-6):
    """keras LayerNormalization(axis=-1): (x - mean) * rsqrt(var + eps) * gamma + beta, biased variance."""
    mean = x.mean(dim=-1, keepdim=True)
    var = ((x - mean) ** 2).mean(dim=-1, keepdim=True)
    inv = torch.rsqrt(var + eps) * gamma
    return x * inv + (beta - mean * inv)


def conditioner_forward(p: Dict[str, torch.Tensor], idx, prefix, down_depth, stride, residual_depth,
                        dilation_factor, reverse_dilation=False, dilation_cycle=None, eps=1e-6):
    """ConditionerNet.call (conditioners.py:74-91): (N, L) codes -> (N, L * stride^down_depth, width)."""
    x = p[f"{prefix}/embedding/embeddings"][torch.as_tensor(idx)]
    b = f"{prefix}/block"
    x = conv1d(x, p[f"{b}/pre/kernel"], p[f"{b}/pre/bias"], 1, 1)          # encdec.py:60
    dil = dilations(residual_depth, dilation_factor, reverse_dilation, dilation_cycle)
    for i in range(down_depth):
        for j, d in enumerate(dil):                                          # resnet.py:7-29
            pa, pb = f"{b}/res{i}/rb{j}/conv_a", f"{b}/res{i}/rb{j}/conv_b"
            h = conv1d(F.relu(x), p[f"{pa}/kernel"], p[f"{pa}/bias"], 1, d)
            x = x + conv1d(F.relu(h), p[f"{pb}/kernel"], p[f"{pb}/bias"], 1, 1)
        x = conv1d_transpose(x, p[f"{b}/up{i}/kernel"], p[f"{b}/up{i}/bias"], stride)  # encdec.py:67-68
    return layer_norm(x, p[f"{prefix}/layer_norm/gamma"], p[f"{prefix}/layer_norm/beta"], eps)
