"""CPU restatement (torch, fp64 by default) of the reference's factorized-attention prior. TEST INFRASTRUCTURE ONLY.

Follows:
  src/transformer/multi_head_attention.py:27-30    create_look_ahead_mask                -> look_ahead_mask
  src/transformer/multi_head_attention.py:62-95    PositionalEmbedding                   -> embed (pos rows [:T])
  keras 2.7 layers.MultiHeadAttention (factorized_attention.py:39-40; query/key/value EinsumDense
      'abc,cde->abde', query * 1/sqrt(key_dim), softmax with (1 - mask) * -1e9, output EinsumDense
      'abcd,cde->abe')                                                                    -> mha
  src/transformer/factorized_attention.py:53-72    FactorizedAttention.call (causal qkv conv, split, proj)
  src/transformer/factorized_attention.py:74-141   row_attn       -> row_attn
  src/transformer/factorized_attention.py:210-286  col_attn       -> col_attn
  src/transformer/factorized_attention.py:308-388  prev_row_attn  -> prev_row_attn
  src/transformer/transformer.py:12-60             ResidualAttnBlock -> res_attn_block
  src/transformer/transformer.py:63-115            FactorizedTransformer (attn_stacks 0: row/col, 1: row/col/prev)
  src/autoregressive/autoregressive_fmha.py:109-160  FMHABasedAutoregressiveModel.call  -> model_forward
  src/autoregressive/autoregressive_fmha.py:162-240  sample (Gumbel noise, argmax)         -> sample_full_recompute
  autoregressive.py:189-212                        loss_function / accuracy_function    -> ce_loss, accuracy
  prior.py:241-335                                 Prior.train_step (teacher forcing, Adam) -> train_step
Dropout: TF's dropout RNG cannot be replayed, so the masks are explicit multipliers (0 or 1/(1-rate)) passed in
(`drop`); the GPU tests read the product's counter-based masks back and hand them over, and test the masks'
statistics separately. Without masks dropout is the identity (rate 0, or training=False).
Parity unpinned: TensorFlow is not importable and the reference holds no fixtures for the prior. The oracle is
pinned by the reference's own sampling-consistency check (factorized_attention.py:446-462: every prefix call
equals the full call at those positions, to 1e-6) and by hand-derived known answers (tests/test_oracle_prior.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from oracle.conditioner_ref import layer_norm


@dataclass
class PriorConfig:
    bins: int = 2048          # target_vocab_size (the VQ-VAE codebook size); start token = bins - 1
    ctx: int = 8192           # context_length (tokens)
    width: int = 128          # d_model
    depth: int = 6
    heads: int = 2
    blocks: int = 4
    attn_stacks: int = 1      # 1: row, col, prev-row (prior.py:414); 0: row, col
    m_attn: float = 0.25
    m_mlp: float = 1.0

    @property
    def attn_width(self) -> int:
        return int(self.width * self.m_attn)

    @property
    def head_dim(self) -> int:
        return self.attn_width // self.heads

    @property
    def block_len(self) -> int:
        return self.ctx // self.blocks

    def attn_func(self, layer: int) -> int:
        """transformer.py:82-86."""
        return [0, 1][layer % 2] if self.attn_stacks == 0 else [0, 1, 2][layer % 3]


def param_specs(cfg: PriorConfig, prefix: str = "prior") -> List[Tuple[str, Tuple[int, ...], str]]:
    """Parameters in the product's ParamStore order / Keras layouts: (name, shape, keras initializer)."""
    W, w, H, hd = cfg.width, cfg.attn_width, cfg.heads, cfg.head_dim
    s = [(f"{prefix}/x_embedding/embeddings", (cfg.bins, W), "uniform"),
         (f"{prefix}/pos_embedding/embeddings", (cfg.ctx, W), "uniform")]
    for l in range(cfg.depth):
        b = f"{prefix}/layer{l}"
        s += [(f"{b}/ln1/gamma", (W,), "ones"), (f"{b}/ln1/beta", (W,), "zeros"),
              (f"{b}/qkv/kernel", (3, W, 3 * w), "glorot_uniform"), (f"{b}/qkv/bias", (3 * w,), "zeros")]
        for n in ("query", "key", "value"):
            s += [(f"{b}/mha/{n}/kernel", (w, H, hd), "glorot_uniform"), (f"{b}/mha/{n}/bias", (H, hd), "zeros")]
        s += [(f"{b}/mha/out/kernel", (H, hd, w), "glorot_uniform"), (f"{b}/mha/out/bias", (w,), "zeros"),
              (f"{b}/proj/kernel", (w, W), "glorot_uniform"), (f"{b}/proj/bias", (W,), "zeros"),
              (f"{b}/ln2/gamma", (W,), "ones"), (f"{b}/ln2/beta", (W,), "zeros"),
              (f"{b}/mlp/kernel", (W, int(W * cfg.m_mlp)), "glorot_uniform"),
              (f"{b}/mlp/bias", (int(W * cfg.m_mlp),), "zeros")]
    s += [(f"{prefix}/out/kernel", (W, cfg.bins), "glorot_uniform"), (f"{prefix}/out/bias", (cfg.bins,), "zeros")]
    return s


def keras_fans(shape) -> Tuple[int, int]:
    """keras initializers _compute_fans (2.7): 2-D (in, out); N-D receptive field = prod(shape[:-2])."""
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[0], shape[1]
    rf = int(np.prod(shape[:-2]))
    return shape[-2] * rf, shape[-1] * rf


def init_params(cfg: PriorConfig, seed: int = 1, prefix: str = "prior") -> Dict[str, np.ndarray]:
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape, init in param_specs(cfg, prefix):
        if init == "glorot_uniform":
            fi, fo = keras_fans(shape)
            lim = math.sqrt(6.0 / (fi + fo))
            out[name] = rng.uniform(-lim, lim, size=shape).astype(np.float32)
        elif init == "uniform":
            out[name] = rng.uniform(-0.05, 0.05, size=shape).astype(np.float32)
        elif init == "ones":
            out[name] = np.ones(shape, np.float32)
        else:
            out[name] = np.zeros(shape, np.float32)
    return out


def look_ahead_mask(q_len: int, k_len: int, dtype=torch.float64):
    """multi_head_attention.py:27-30: band_part(ones, -1, 0) (1 = attend)."""
    return torch.tril(torch.ones(q_len, k_len, dtype=dtype))


def causal_conv(x, W, b):
    """layers.Conv1D(filters, 3, padding='causal') (factorized_attention.py:36): y[t] = sum_k x[t-2+k] W[k] + b."""
    K = W.shape[0]
    xp = torch.nn.functional.pad(x, (0, 0, K - 1, 0))
    T = x.shape[1]
    return sum(xp[:, k:k + T] @ W[k] for k in range(K)) + b


def mha(p, pre, q_in, k_in, v_in, mask=None):
    """keras MultiHeadAttention(num_heads, key_dim, value_dim) on (N, Tq, w) / (N, Tk, w): returns (N, Tq, w)."""
    q = torch.einsum("abc,cde->abde", q_in, p[f"{pre}/query/kernel"]) + p[f"{pre}/query/bias"]
    k = torch.einsum("abc,cde->abde", k_in, p[f"{pre}/key/kernel"]) + p[f"{pre}/key/bias"]
    v = torch.einsum("abc,cde->abde", v_in, p[f"{pre}/value/kernel"]) + p[f"{pre}/value/bias"]
    q = q * (1.0 / math.sqrt(q.shape[-1]))
    s = torch.einsum("aecd,abcd->acbe", k, q)                      # (N, H, Tq, Tk)
    if mask is not None:
        s = s + (1.0 - mask) * -1e9
    a = torch.softmax(s, dim=-1)
    o = torch.einsum("acbe,aecd->abcd", a, v)                     # (N, Tq, H, hd)
    return torch.einsum("abcd,cde->abe", o, p[f"{pre}/out/kernel"]) + p[f"{pre}/out/bias"]


def row_attn(p, pre, q, k, v, l):
    """factorized_attention.py:74-141 (training: trail 0; sampling: a causal partial last block)."""
    N, L, D = k.shape
    trail, nb = L % l, L // l
    outs = []
    if nb > 0:
        qc, kc, vc = (t[:, :nb * l].reshape(N * nb, l, D) for t in (q, k, v))
        outs.append(mha(p, pre, qc, kc, vc, look_ahead_mask(l, l, q.dtype)).reshape(N, nb * l, D))
    if trail > 0:
        outs.append(mha(p, pre, q[:, -trail:], k[:, -trail:], v[:, -trail:], look_ahead_mask(trail, trail, q.dtype)))
    return torch.cat(outs, dim=1)


def col_attn(p, pre, q, k, v, l):
    """factorized_attention.py:210-286: position j of block b attends positions j of blocks 0..b."""
    N, L, D = k.shape
    trail, nb = L % l, L // l
    outs = []
    if nb > 0:
        def cols(t):
            return t[:, :nb * l].reshape(N, nb, l, D).transpose(1, 2).reshape(N * l, nb, D)
        o = mha(p, pre, cols(q), cols(k), cols(v), look_ahead_mask(nb, nb, q.dtype))
        outs.append(o.reshape(N, l, nb, D).transpose(1, 2).reshape(N, nb * l, D))
    if trail > 0:
        def cur(t):
            prev = t[:, :nb * l].reshape(N, nb, l, D)[:, :, :trail]                  # (N, nb, trail, D)
            c = torch.cat([prev, t[:, -trail:].unsqueeze(1)], dim=1)                 # (N, nb+1, trail, D)
            return c.transpose(1, 2).reshape(N * trail, nb + 1, D)
        qc = q[:, -trail:].reshape(N * trail, 1, D)
        outs.append(mha(p, pre, qc, cur(k), cur(v), None).reshape(N, trail, D))
    return torch.cat(outs, dim=1)


def prev_row_attn(p, pre, q, k, v, l):
    """factorized_attention.py:308-388: block b attends every position of block b-1 (a zero block before b=0)."""
    N, L, D = k.shape
    trail, nb = L % l, L // l
    outs = []
    if nb > 0:
        qc = q[:, :nb * l].reshape(N * nb, l, D)
        def shifted(t):
            t4 = t[:, :nb * l].reshape(N, nb, l, D)
            t4 = torch.cat([torch.zeros_like(t4[:, :1]), t4[:, :-1]], dim=1)
            return t4.reshape(N * nb, l, D)
        outs.append(mha(p, pre, qc, shifted(k), shifted(v), None).reshape(N, nb * l, D))
    if trail > 0:
        if nb > 0:
            kc, vc = k[:, (nb - 1) * l:nb * l], v[:, (nb - 1) * l:nb * l]
        else:
            kc = torch.zeros(N, l, D, dtype=k.dtype)
            vc = torch.zeros(N, l, D, dtype=v.dtype)
        outs.append(mha(p, pre, q[:, -trail:], kc, vc, None))
    return torch.cat(outs, dim=1)


ATTN = {0: row_attn, 1: col_attn, 2: prev_row_attn}


def res_attn_block(p, pre, x, attn_type, l, drop=None):
    """transformer.py:35-60 with FactorizedAttention.call (factorized_attention.py:53-72). drop: the attention
    output's keras Dropout as an explicit multiplier (0 or 1/(1-rate)), factorized_attention.py:51,72."""
    a = layer_norm(x, p[f"{pre}/ln1/gamma"], p[f"{pre}/ln1/beta"])
    qkv = causal_conv(a, p[f"{pre}/qkv/kernel"], p[f"{pre}/qkv/bias"])
    q, k, v = qkv.chunk(3, dim=-1)
    o = ATTN[attn_type](p, f"{pre}/mha", q, k, v, l)
    res1 = o @ p[f"{pre}/proj/kernel"] + p[f"{pre}/proj/bias"]
    if drop is not None:
        res1 = res1 * drop
    h = layer_norm(x + res1, p[f"{pre}/ln2/gamma"], p[f"{pre}/ln2/beta"])
    res2 = h @ p[f"{pre}/mlp/kernel"] + p[f"{pre}/mlp/bias"]
    return res2 + res1 + x


def embed(p, cfg: PriorConfig, tokens, prefix="prior", y_cond=None, x_cond=None, drop=None):
    """autoregressive_fmha.py:119-151 (pos_emb=True). drop: the embedding Dropout (:139) as an explicit
    multiplier, None = identity."""
    x = p[f"{prefix}/x_embedding/embeddings"][torch.as_tensor(tokens)]
    if y_cond is not None:
        x = torch.cat([torch.as_tensor(y_cond, dtype=x.dtype), x[:, 1:]], dim=1)
    x = x * math.sqrt(cfg.width)
    x = x + p[f"{prefix}/pos_embedding/embeddings"][:x.shape[1]].unsqueeze(0)
    if drop is not None:
        x = x * drop
    if x_cond is not None:
        x = x + torch.as_tensor(x_cond, dtype=x.dtype)[:, :x.shape[1]]
    return x


def model_forward(p, cfg: PriorConfig, tokens, prefix="prior", y_cond=None, x_cond=None, drop=None):
    """(N, T) tokens -> (N, T, bins) logits. drop: {"emb": mask, "layer{i}": mask} dropout multipliers."""
    drop = drop or {}
    x = embed(p, cfg, tokens, prefix, y_cond, x_cond, drop.get("emb"))
    for layer in range(cfg.depth):
        x = res_attn_block(p, f"{prefix}/layer{layer}", x, cfg.attn_func(layer), cfg.block_len,
                           drop.get(f"layer{layer}"))
    return x @ p[f"{prefix}/out/kernel"] + p[f"{prefix}/out/bias"]


def ce_loss(target, logits):
    """SparseCategoricalCrossentropy(from_logits=True, reduction=NONE) then reduce_mean (autoregressive.py:189-201)."""
    lse = torch.logsumexp(logits, dim=-1)
    tl = torch.gather(logits, -1, torch.as_tensor(target).unsqueeze(-1)).squeeze(-1)
    return (lse - tl).mean()


def argmax_lowest(x):
    """tf.argmax: first index of the maximum."""
    return torch.argmax(x, dim=-1)  # torch returns the first maximal index as well


def accuracy(target, logits):
    """autoregressive.py:203-212."""
    return (torch.as_tensor(target) == argmax_lowest(logits)).to(logits.dtype).mean()


def shift_right(codes, start_token):
    """prior.py:262-263: pad(codes[:, :-1], [[0,0],[1,0]], constant_values=bins-1)."""
    c = torch.as_tensor(codes)
    return torch.cat([torch.full_like(c[:, :1], start_token), c[:, :-1]], dim=1)


def train_step_grads(p, cfg: PriorConfig, codes, tf_mask, prefix="prior", x_cond=None, labels=None, drop1=None,
                     drop2=None):
    """prior.py:272-300: forward once, argmax -> shifted predictions, mix with the shifted codes where tf_mask
    (= uniform < teacher_force_rate), forward again with gradients. Returns (loss, accuracy, grads, batch_input).
    labels = (table name, y): the LabelConditioner's rows (label_conditioners.py:26-45) replace position 0 and
    are trained with the prior (prior.py:268-271,299). drop1 / drop2: the two passes' dropout multipliers."""
    start = cfg.bins - 1
    latent_input = shift_right(codes, start)

    def ycond(q):
        if labels is None:
            return None
        name, y = labels
        return q[name][torch.as_tensor(y)].unsqueeze(1)

    with torch.no_grad():
        logits0 = model_forward(p, cfg, latent_input, prefix, y_cond=ycond(p), x_cond=x_cond, drop=drop1)
    pred = shift_right(argmax_lowest(logits0), start)
    batch_input = torch.where(torch.as_tensor(tf_mask), pred, latent_input)
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
    logits = model_forward(leaves, cfg, batch_input, prefix, y_cond=ycond(leaves), x_cond=x_cond, drop=drop2)
    loss = ce_loss(codes, logits)
    loss.backward()
    grads = {k: (v.grad if v.grad is not None else torch.zeros_like(v)) for k, v in leaves.items()}
    return float(loss.detach()), float(accuracy(codes, logits.detach())), grads, batch_input


def gumbel_uniform(seed: int, n: int, step: int, k: np.ndarray) -> np.ndarray:
    """The product's counter-based uniform in (0, 1) for (sample n, step, bin k) (vqa_prior.hip prior_uniform):
    splitmix64-style hash of (seed, n, step, k) -> 24 high bits -> (u + 0.5) / 2^24. numpy restatement."""
    M = np.uint64(0xFFFFFFFFFFFFFFFF)

    def sm(x):
        x = (x + np.uint64(0x9E3779B97F4A7C15)) & M
        x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M
        x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M
        return x ^ (x >> np.uint64(31))

    with np.errstate(over="ignore"):
        h = sm(np.uint64(seed))
        h = sm(h ^ np.uint64(n))
        h = sm(h ^ np.uint64(step))
        h = sm(h ^ k.astype(np.uint64))
    u = (h >> np.uint64(40)).astype(np.float64)
    return ((u + 0.5) / float(1 << 24)).astype(np.float32)


def gumbel_noise(seed: int, n: int, step: int, bins: int) -> np.ndarray:
    """-log(-log(U)) in fp32 (the product computes it with the same fp32 formula)."""
    u = gumbel_uniform(seed, n, step, np.arange(bins))
    return (-np.log(-np.log(u.astype(np.float32)))).astype(np.float32)


def sample_full_recompute(p, cfg: PriorConfig, n_samples: int, max_length: int, seed: int, prefix="prior",
                          x_cond=None, y_cond=None):
    """autoregressive_fmha.py:162-240: start token, then max_length steps of a FULL forward over the prefix,
    last-position logits + Gumbel noise (RelaxedOneHotCategorical(1).sample() then argmax = argmax(logits + G)).
    Returns (N, max_length + 1) int64 tokens and the per-step top-2 margins of logits + G."""
    out = torch.full((n_samples, 1), cfg.bins - 1, dtype=torch.int64)
    margins = np.zeros((n_samples, max_length))
    for i in range(max_length):
        logits = model_forward(p, cfg, out, prefix, y_cond=y_cond, x_cond=x_cond)[:, -1]  # (N, bins)
        g = torch.from_numpy(np.stack([gumbel_noise(seed, n, i, cfg.bins) for n in range(n_samples)])).to(logits.dtype)
        z = logits + g
        top2 = torch.topk(z, 2, dim=-1).values
        margins[:, i] = (top2[:, 0] - top2[:, 1]).numpy()
        out = torch.cat([out, argmax_lowest(z).unsqueeze(1)], dim=1)
    return out, margins


def to_torch(params: Dict[str, np.ndarray], dtype=torch.float64) -> Dict[str, torch.Tensor]:
    return {k: torch.from_numpy(np.asarray(v)).to(dtype) for k, v in params.items()}
