"""Factorized-attention prior — drop-in for the reference's prior stack (BASELINE configs 4-5).

Reference classes kept here (same names, constructor arguments and call surface):
  src/transformer/factorized_attention.py:10-72  FactorizedAttention(ctc_len, num_heads, d_model, blocks, attn_func,
                                                   m_attn, drop_out_rate): causal Conv1D(3w, 3) -> split q, k, v ->
                                                   keras MultiHeadAttention(num_heads, key_dim=w/H) core of the
                                                   row (0) / col (1) / prev-row (2) factorization -> Dense(d_model)
  src/transformer/transformer.py:12-60           ResidualAttnBlock: out = mlp(LN2(x + a)) + a + x, a = fmha(LN1(x))
  src/transformer/transformer.py:63-115          FactorizedTransformer (attn_stacks 0: row/col, 1: row/col/prev-row)
  src/autoregressive/autoregressive_fmha.py:13-240  FMHABasedAutoregressiveModel: embedding * sqrt(d) + positional
                                                   embedding (+ x_cond from ConditionerNet), transformer, Dense(bins);
                                                   sample() = Gumbel-max ancestral sampling
  prior.py:102-372                               Prior: train_step with teacher forcing (two forward passes, the
                                                   second mixes the first pass's argmax into the input at
                                                   teacher_force_rate), loss/accuracy trackers, Keras Adam
  src/conditioner/label_conditioners.py:9-48     LabelConditioner (genre Embedding -> the start position)

MI355X path (libvqa, vqa_prior.hip): every linear layer is the MFMA sequence-linear kernel (the causal conv is
its 3-tap form); attention is flash-style on MFMA for the row / prev-row blocks and a register kernel for the
4-long columns; the output Dense is fused with the cross entropy / argmax so the (N, T, bins) logits are never
written; sampling is ONE persistent kernel per batch that walks the positions with a key/value cache instead of
re-running the model on the prefix at every step. All gradients are explicit; weight gradients are fixed-order
partial reductions (deterministic). Dropout uses a counter-based mask (TF's RNG cannot be replayed).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import torch

import vqa_dp
import vqa_lib as V
from conditioners import ConditionerNet
from vqa_layers import CKPT_VERSION, ParamStore, checkpoint_layout
from vqa_metrics import Mean
from vqa_module import keras_evaluate
from vqa_optim import Adam


def create_look_ahead_mask(q_len, k_len):
    """multi_head_attention.py:27-30 (1 = attend)."""
    return torch.tril(torch.ones(q_len, k_len))


def positional_encoding(position, d_model):
    """multi_head_attention.py:33-59: (1, position, d_model) sinusoid table (fp32)."""
    pos = np.arange(position)[:, None]
    i = np.arange(d_model)[None, :]
    ang = pos / np.power(10000, (2 * (i // 2)) / np.float32(d_model))
    ang[:, 0::2] = np.sin(ang[:, 0::2])
    ang[:, 1::2] = np.cos(ang[:, 1::2])
    return ang[None].astype(np.float32)


ATTN_NAMES = {0: "row", 1: "col", 2: "prev row"}


class FactorizedAttention:
    def __init__(self, ctc_len, num_heads, d_model, blocks, attn_func=0, m_attn=0.25, drop_out_rate=0.0, **kwargs):
        self.width = int(d_model * m_attn)
        assert self.width % num_heads == 0
        self.num_heads, self.ctx_len, self.blocks, self.d_model = num_heads, ctc_len, blocks, d_model
        assert self.ctx_len % blocks == 0
        self.block_len = self.ctx_len // blocks
        self.attn_func, self.attn_type = attn_func, ATTN_NAMES[attn_func]
        self.rate = drop_out_rate
        self.head_dim = self.width // num_heads

    def build(self, store: ParamStore, prefix: str):
        w, H, hd, d = self.width, self.num_heads, self.head_dim, self.d_model
        self.prefix, self.store = prefix, store
        store.add(f"{prefix}/qkv/kernel", (3, d, 3 * w), "glorot_uniform")
        store.add(f"{prefix}/qkv/bias", (3 * w,), "zeros")
        for n in ("query", "key", "value"):
            store.add(f"{prefix}/mha/{n}/kernel", (w, H, hd), "glorot_uniform")
            store.add(f"{prefix}/mha/{n}/bias", (H, hd), "zeros")
        store.add(f"{prefix}/mha/out/kernel", (H, hd, w), "glorot_uniform")
        store.add(f"{prefix}/mha/out/bias", (w,), "zeros")
        store.add(f"{prefix}/proj/kernel", (w, d), "glorot_uniform")
        store.add(f"{prefix}/proj/bias", (d,), "zeros")

    def p(self, name):
        return self.store.view(f"{self.prefix}/{name}")

    def g(self, name):
        return self.store.grad_view(f"{self.prefix}/{name}")


class ResidualAttnBlock:
    def __init__(self, ctc_len, num_heads, d_model, blocks, attn_func=0, m_attn=0.25, m_mlp=1.0, rate=0.1, **kwargs):
        self.d_model, self.attn_func = d_model, attn_func
        self.fmha = FactorizedAttention(ctc_len, num_heads, d_model, blocks, attn_func=attn_func, m_attn=m_attn,
                                        drop_out_rate=rate)
        self.mlp_width = int(d_model * m_mlp)
        if self.mlp_width != d_model:
            raise ValueError("m_mlp != 1 changes the residual width (transformer.py:54-56 adds mlp output to x)")

    def build(self, store: ParamStore, prefix: str):
        d = self.d_model
        self.prefix, self.store = prefix, store
        store.add(f"{prefix}/ln1/gamma", (d,), "ones")
        store.add(f"{prefix}/ln1/beta", (d,), "zeros")
        self.fmha.build(store, prefix)
        store.add(f"{prefix}/ln2/gamma", (d,), "ones")
        store.add(f"{prefix}/ln2/beta", (d,), "zeros")
        store.add(f"{prefix}/mlp/kernel", (d, self.mlp_width), "glorot_uniform")
        store.add(f"{prefix}/mlp/bias", (self.mlp_width,), "zeros")

    # -------------------------------------------------------------- weight images (vqa_seqlin_prep)
    def prep_descs(self, cdt, device, bwd):
        """(w, out, taps, K, N, wtrans) of every linear map: forward images, and with bwd the transposed images
        of the data gradients. The buffers persist; their contents are refreshed once per step."""
        f, st, pre, d, w = self.fmha, self.store, self.prefix, self.d_model, self.fmha.width
        maps = {"qkv": (f"{pre}/qkv/kernel", 3, d, 3 * w), "query": (f"{pre}/mha/query/kernel", 1, w, w),
                "key": (f"{pre}/mha/key/kernel", 1, w, w), "value": (f"{pre}/mha/value/kernel", 1, w, w),
                "out": (f"{pre}/mha/out/kernel", 1, w, w), "proj": (f"{pre}/proj/kernel", 1, w, d),
                "mlp": (f"{pre}/mlp/kernel", 1, d, self.mlp_width)}
        if not hasattr(self, "wp") or self._wp_dtype != cdt:
            self.wp, self._wp_dtype = {}, cdt
        out = []
        for name, (pname, taps, K, N) in maps.items():
            for tr in ((False, True) if bwd else (False,)):
                key = name + ("_T" if tr else "")
                Ki, Ni = (N, K) if tr else (K, N)
                if key not in self.wp:
                    self.wp[key] = torch.empty(taps, Ni, Ki, dtype=cdt, device=device)
                # forward: Wv = W (K, N); transposed (data gradient): Wv[k=out][n=in] = W[n][k] -> wtrans
                out.append((st.view(pname), self.wp[key], taps, Ki, Ni, tr))
        return out

    # -------------------------------------------------------------- forward / backward on the device
    def forward(self, x, T, training, save, seed, salt, counter=None, row0=0):
        """x (N, T, d) -> (N, T, d). save: keep what backward needs (layer input, qkv, heads, lse, o32, x1).
        row0: the global index of x's first (sequence, position) row — the dropout mask's key under data
        parallelism (rank * N * T), so every rank draws its slice of the single-process mask."""
        f, cdt, eps = self.fmha, x.dtype, 1e-6
        N = x.shape[0]
        w = f.width
        qkv = torch.empty(N, T, 3 * w, dtype=cdt, device=x.device)
        wp = self.wp
        g1, b1 = self.store.view(f"{self.prefix}/ln1/gamma"), self.store.view(f"{self.prefix}/ln1/beta")
        fused = V.seqlin_fused_ln_ok(x, x.shape[-1])  # LayerNorm inside the consumer's row loads (bit-identical)
        if fused:
            V.seqlin_fwd_ln_prepped(x, g1, b1, eps, wp["qkv"], f.p("qkv/bias"), qkv, T, taps=3, dir=-1)
        else:
            a = torch.empty_like(x)
            V.layernorm_fwd(x, g1, b1, a, eps)
            V.seqlin_fwd_prepped(a, wp["qkv"], f.p("qkv/bias"), qkv, T, taps=3, dir=-1)
        heads = []
        for j, n in enumerate(("query", "key", "value")):
            h = torch.empty(N, T, w, dtype=cdt, device=x.device)
            V.seqlin_fwd_prepped(qkv[..., j * w:(j + 1) * w], wp[n], f.p(f"mha/{n}/bias"), h, T)
            heads.append(h)
        qh, kh, vh = heads
        oh = torch.empty_like(qh)
        lse = torch.empty(N, T, f.num_heads, dtype=torch.float32, device=x.device)
        V.attn_fwd(qh, kh, vh, oh, lse, f.attn_func, f.block_len, f.num_heads, 1.0 / math.sqrt(f.head_dim),
                   vbias=f.p("mha/value/bias"))
        o32 = torch.empty_like(qh)
        V.seqlin_fwd_prepped(oh, wp["out"], f.p("mha/out/bias"), o32, T)
        x1 = torch.empty_like(x)
        drop = training and f.rate > 0
        if drop:
            V.seqlin_fwd_prepped(o32, wp["proj"], f.p("proj/bias"), x1, T)
            V.dropout_(x1, f.rate, seed, salt, counter, elem_offset=row0 * x.shape[-1])
            V.axpy(x1, x, x1)
        else:
            V.seqlin_fwd_prepped(o32, wp["proj"], f.p("proj/bias"), x1, T, residual=x)
        g2, b2 = self.store.view(f"{self.prefix}/ln2/gamma"), self.store.view(f"{self.prefix}/ln2/beta")
        out = torch.empty_like(x)
        if fused:
            V.seqlin_fwd_ln_prepped(x1, g2, b2, eps, wp["mlp"], self.store.view(f"{self.prefix}/mlp/bias"), out, T,
                                    residual=x1)
        else:
            h2 = torch.empty_like(x)
            V.layernorm_fwd(x1, g2, b2, h2, eps)
            V.seqlin_fwd_prepped(h2, wp["mlp"], self.store.view(f"{self.prefix}/mlp/bias"), out, T, residual=x1)
        self._saved = (x, qkv, qh, kh, vh, oh, lse, o32, x1, drop, seed, salt, counter, row0) if save else None
        return out

    def backward(self, dout, T, deferred, post_adds):
        """dout = dL/d(out) -> dL/dx; weight gradients into the store (deferred partial reductions)."""
        x, qkv, qh, kh, vh, oh, lse, o32, x1, drop, seed, salt, counter, row0 = self._saved
        self._saved = None
        f, st, pre, eps = self.fmha, self.store, self.prefix, 1e-6
        N, w, cdt = x.shape[0], f.width, x.dtype
        # mlp: out = mlp(LN2(x1)) + x1
        h2 = torch.empty_like(x)
        V.layernorm_fwd(x1, st.view(f"{pre}/ln2/gamma"), st.view(f"{pre}/ln2/beta"), h2, eps)
        dh2 = torch.empty_like(x)
        wp = self.wp
        V.seqlin_fwd_prepped(dout, wp["mlp_T"], None, dh2, T)
        V.seqlin_wgrad(h2, dout, st.grad_view(f"{pre}/mlp/kernel"), st.grad_view(f"{pre}/mlp/bias"), T,
                       deferred=deferred)
        dx1 = torch.empty_like(x)
        V.layernorm_bwd(x1, dh2, st.view(f"{pre}/ln2/gamma"), dx1, st.grad_view(f"{pre}/ln2/gamma"),
                        st.grad_view(f"{pre}/ln2/beta"), eps, deferred)
        V.axpy(dx1, dout, dx1)
        # x1 = x + dropout(proj(o32))
        dres1 = dx1
        if drop:
            dres1 = dx1.clone()
            V.dropout_(dres1, f.rate, seed, salt, counter, elem_offset=row0 * x.shape[-1])
        do32 = torch.empty_like(qh)
        V.seqlin_fwd_prepped(dres1, wp["proj_T"], None, do32, T)
        V.seqlin_wgrad(o32, dres1, f.g("proj/kernel"), f.g("proj/bias"), T, deferred=deferred)
        doh = torch.empty_like(qh)
        V.seqlin_fwd_prepped(do32, wp["out_T"], None, doh, T)
        V.seqlin_wgrad(oh, do32, f.g("mha/out/kernel"), f.g("mha/out/bias"), T, deferred=deferred)
        dqh, dkh, dvh = torch.empty_like(qh), torch.empty_like(qh), torch.empty_like(qh)
        dsum = torch.empty(N, T, f.num_heads, dtype=torch.float32, device=x.device)
        V.attn_bwd(qh, kh, vh, oh, lse, doh, dsum, dqh, dkh, dvh, f.attn_func, f.block_len, f.num_heads,
                   1.0 / math.sqrt(f.head_dim))
        if f.attn_func == 2:
            # the zero block of block 0: its values are the value bias, d(bias) += sum of dO over block 0 —
            # per-position sums over the batch, then a fixed-order reduction of those rows (deferred)
            tmp = torch.empty(f.block_len, w, dtype=torch.float32, device=x.device)
            V.colsum(doh, tmp, N, T * w, f.block_len * w)
            extra = torch.empty(w, dtype=torch.float32, device=x.device)
            deferred.add(V.PartialsDesc(tmp.data_ptr(), extra.data_ptr(), None, f.block_len, w, w, 0), tmp)
            post_adds.append((f.g("mha/value/bias").view(-1), extra))
        dqkv = torch.empty_like(qkv)
        for j, (n, dh) in enumerate((("query", dqh), ("key", dkh), ("value", dvh))):
            V.seqlin_fwd_prepped(dh, wp[f"{n}_T"], None, dqkv[..., j * w:(j + 1) * w], T)
            V.seqlin_wgrad(qkv[..., j * w:(j + 1) * w], dh, f.g(f"mha/{n}/kernel"), f.g(f"mha/{n}/bias"), T,
                           deferred=deferred)
        a = torch.empty_like(x)
        V.layernorm_fwd(x, st.view(f"{pre}/ln1/gamma"), st.view(f"{pre}/ln1/beta"), a, eps)
        da = torch.empty_like(x)
        V.seqlin_fwd_prepped(dqkv, wp["qkv_T"], None, da, T, taps=3, dir=1)
        V.seqlin_wgrad(a, dqkv, f.g("qkv/kernel"), f.g("qkv/bias"), T, taps=3, deferred=deferred)
        dx = torch.empty_like(x)
        V.layernorm_bwd(x, da, st.view(f"{pre}/ln1/gamma"), dx, st.grad_view(f"{pre}/ln1/gamma"),
                        st.grad_view(f"{pre}/ln1/beta"), eps, deferred)
        V.axpy(dx, dx1, dx)
        return dx

    def layer_desc(self):
        st, pre = self.store, self.prefix
        v = lambda n: st.view(f"{pre}/{n}").data_ptr()
        return V.PriorLayerDesc(v("ln1/gamma"), v("ln1/beta"), v("qkv/kernel"), v("qkv/bias"), v("mha/query/kernel"),
                                v("mha/query/bias"), v("mha/key/kernel"), v("mha/key/bias"), v("mha/value/kernel"),
                                v("mha/value/bias"), v("mha/out/kernel"), v("mha/out/bias"), v("proj/kernel"),
                                v("proj/bias"), v("ln2/gamma"), v("ln2/beta"), v("mlp/kernel"), v("mlp/bias"),
                                self.attn_func)


class FactorizedTransformer:
    def __init__(self, ctc_len, num_heads, depth, d_model, blocks, attn_stacks, m_attn=0.25, m_mlp=1.0, rate=0.1,
                 **kwargs):
        self.d_model, self.depth = d_model, depth
        self.attn_func = {0: lambda d: [0, 1][d % 2], 1: lambda d: [0, 1, 2][d % 3]}[attn_stacks]
        self.layers = [ResidualAttnBlock(ctc_len, num_heads, d_model, blocks, attn_func=self.attn_func(i),
                                         m_attn=m_attn, m_mlp=m_mlp, rate=rate) for i in range(depth)]

    def build(self, store, prefix):
        for i, ly in enumerate(self.layers):
            ly.build(store, f"{prefix}/layer{i}")


class LabelConditioner:
    """label_conditioners.py:9-48: genre Embedding(genre_bins, width) -> (N, 1, width)."""

    def __init__(self, genre_bins, width, **kwargs):
        self.genre_bins, self.model = genre_bins, width

    def build(self, store, prefix):
        self.store, self.name = store, store.add(f"{prefix}/genre_embedding/embeddings", (self.genre_bins, self.model),
                                                 "uniform")

    def __call__(self, y, training=False, **kwargs):
        y = torch.as_tensor(y, device=self.store.flat.device).long().reshape(-1)
        return self.store.view(self.name)[y].unsqueeze(1)


class FMHABasedAutoregressiveModel:
    """autoregressive_fmha.py:13-240 on libvqa. dtype 'fp32' (parity) or 'bf16' (activations; fp32 weights)."""

    def __init__(self, target_vocab_size, width, depth, blocks, m_attn=0.25, m_mlp=1.0, heads=1, attn_stacks=1,
                 maximum_pos_encoding=5000, drop_out_rate=0.1, context_length=None, zq_shapes=None, level=0, levels=3,
                 pos_emb=True, downs=None, strides=None, cond_kwargs=None, dtype="fp32", device="cuda", seed=1,
                 store: Optional[ParamStore] = None, prefix="prior", grad_extra: int = 0, label_bins=None, **kwargs):
        self.context_length = int(np.prod(context_length))
        self.bins, self.d_model, self.depth = target_vocab_size, width, depth
        self.heads, self.blocks = heads, blocks
        self.use_pos_embedding = pos_emb
        self.levels, self.level, self.cond_level = levels, level, level + 1
        self.rate = drop_out_rate
        self.start_token = self.bins - 1
        self.cdt = torch.bfloat16 if dtype == "bf16" else torch.float32
        self.device = torch.device(device)
        self.cond_downsample_rate = (strides[self.cond_level] ** downs[self.cond_level]
                                     if (strides is not None and self.level != levels - 1) else None)
        self.transformer = FactorizedTransformer(self.context_length, heads, depth, width, blocks, attn_stacks,
                                                 m_attn=m_attn, m_mlp=m_mlp, rate=drop_out_rate)
        self.conditioner = None
        if self.cond_level != levels and cond_kwargs is not None:
            self.conditioner = ConditionerNet(cond_shape=zq_shapes[self.cond_level], bins=self.bins,
                                              embed_width=self.d_model, down_depth=downs[self.cond_level],
                                              stride=strides[self.cond_level], **cond_kwargs)
        own = store is None
        self.store = store if store is not None else ParamStore()
        self.prefix = prefix
        st = self.store
        self.emb_name = st.add(f"{prefix}/x_embedding/embeddings", (self.bins, width), "uniform")
        self.pos_name = (st.add(f"{prefix}/pos_embedding/embeddings", (self.context_length, width), "uniform")
                         if pos_emb else None)
        self.transformer.build(st, prefix)
        self.out_kernel = st.add(f"{prefix}/out/kernel", (width, self.bins), "glorot_uniform")
        self.out_bias = st.add(f"{prefix}/out/bias", (self.bins,), "zeros")
        if self.conditioner is not None:
            self.conditioner.build(st, f"{prefix}/conditioner", width, self.cdt)
        # prior.py:154-157: the Prior's LabelConditioner (genre embedding -> position 0), in the same store so
        # that Adam and the data-parallel bucket cover it
        self.label_conditioner = None
        if label_bins is not None:
            self.label_conditioner = LabelConditioner(label_bins, width)
            self.label_conditioner.build(st, "label_conditioner")
        if own:
            # the gradient buffer is the head of the data-parallel bucket: grad_extra trailing slots for scalars
            st.materialize(self.device, grad_buffer=torch.zeros(st.size + grad_extra, device=self.device), seed=seed)
        self._pos_table = None
        if not pos_emb:
            self._pos_table = torch.from_numpy(positional_encoding(maximum_pos_encoding, width)[0]).to(self.device)
        self._counter = 0

    # -------------------------------------------------------------- pieces
    def _pos(self):
        return self.store.view(self.pos_name) if self.use_pos_embedding else self._pos_table

    def _wt(self, dtype):
        wt = torch.empty(self.bins, self.d_model, dtype=dtype, device=self.device)
        V.head_wt(self.store.view(self.out_kernel), wt)
        return wt

    def _embed(self, tokens, training, x_cond=None, y_cond=None, seed=0, counter=None, row0=0):
        N, T = tokens.shape
        x = torch.empty(N, T, self.d_model, dtype=self.cdt, device=self.device)
        V.prior_embed_fwd(self.store.view(self.emb_name), self._pos(), tokens, x, math.sqrt(self.d_model),
                          ycond=y_cond, xcond=x_cond, rate=self.rate if training else 0.0, seed=seed, counter=counter,
                          elem_offset=row0 * self.d_model)
        return x

    def prep_weights(self, bwd=False):
        """Refresh every layer's weight images in one launch (vqa_seqlin_prep): forward, and with bwd the
        transposed images of the data gradients."""
        descs = []
        for ly in self.transformer.layers:
            descs += ly.prep_descs(self.cdt, self.device, bwd)
        V.seqlin_prep(descs, self.cdt)

    def hidden(self, tokens, training=False, x_cond=None, y_cond=None, save=False, seed=0, counter=None,
               prepped=False, row0=0):
        """Embedding + transformer: (N, T) tokens -> (N, T, d) final hidden state (the head's input). row0: the
        global index of the first (sequence, position) row (data parallel: rank * N * T) — the dropout masks' key."""
        if not prepped:
            self.prep_weights(bwd=False)
        tokens = tokens.contiguous()
        N, T = tokens.shape
        if self.use_pos_embedding and T > self.context_length:
            raise ValueError(f"sequence of {T} > context length {self.context_length}")
        # the embedding kernel reads x_cond[n, t] (n < N, t < T) and y_cond[n]: check before passing pointers
        if x_cond is not None and (x_cond.dim() != 3 or x_cond.shape[0] != N or x_cond.shape[1] < T
                                   or x_cond.shape[2] != self.d_model):
            raise ValueError(f"x_cond shape {tuple(x_cond.shape)}: expected ({N}, >= {T}, {self.d_model})")
        if x_cond is not None and x_cond.shape[1] != T:
            x_cond = x_cond[:, :T].contiguous()
        if y_cond is not None and tuple(y_cond.shape) != (N, self.d_model):
            raise ValueError(f"y_cond shape {tuple(y_cond.shape)}: expected ({N}, {self.d_model})")
        x = self._embed(tokens, training, x_cond, y_cond, seed, counter, row0)
        for i, ly in enumerate(self.transformer.layers):
            x = ly.forward(x, T, training, save, seed, 1000 + i, counter, row0)
        return x

    def _cond(self, x_cond, save=False):
        if x_cond is None:
            return None
        x_cond = torch.as_tensor(x_cond, device=self.device)
        if x_cond.dim() == 3:  # already up-sampled (autoregressive_fmha.py:145-148)
            return x_cond.to(self.cdt).contiguous()
        return self.conditioner.forward(x_cond.long().contiguous(), save=save)

    # -------------------------------------------------------------- Keras-like call / sample
    def __call__(self, x, training=False, x_cond=None, y_cond=None):
        """autoregressive_fmha.py:109-160 -> ((N, T, bins) fp32 logits, {}). Logits are materialised here (the
        training step never does): 128-wide vocab slices of the head as sequence-linear launches."""
        tokens = torch.as_tensor(x, device=self.device).long()
        with torch.no_grad():
            h = self.hidden(tokens, training, self._cond(x_cond), self._ycond(y_cond))
            N, T = tokens.shape
            # the vocabulary zero-padded to a multiple of 16 (the sequence-linear kernel's output tile)
            Vp = -(-self.bins // 16) * 16
            wt32 = torch.zeros(Vp, self.d_model, dtype=torch.float32, device=self.device)
            V.head_wt(self.store.view(self.out_kernel), wt32[:self.bins])
            hf = h.float().contiguous()
            logits = torch.empty(N, T, Vp, dtype=torch.float32, device=self.device)
            b = torch.zeros(Vp, dtype=torch.float32, device=self.device)
            b[:self.bins] = self.store.view(self.out_bias)
            for v0 in range(0, Vp, 128):
                n = min(128, Vp - v0)
                V.seqlin_fwd(hf, wt32[v0:v0 + n], b[v0:v0 + n], logits[..., v0:v0 + n], T, wtrans=True)
        return (logits[..., :self.bins].contiguous() if Vp != self.bins else logits), {}

    call = __call__

    def _ycond(self, y_cond, n=None):
        """(N, d_model) fp32 label embeddings for position 0 (label_conditioners.py:26-45 gives (N, 1, d_model));
        n: the number of sequences it must cover (the kernels read one row per sequence)."""
        if y_cond is None:
            return None
        yc = torch.as_tensor(y_cond, device=self.device, dtype=torch.float32)
        if yc.shape[-1] != self.d_model or yc.numel() % self.d_model:
            raise ValueError(f"y_cond shape {tuple(yc.shape)}: last dimension must be {self.d_model}")
        yc = yc.reshape(-1, self.d_model).contiguous()
        if n is not None and yc.shape[0] != n:
            raise ValueError(f"y_cond has {yc.shape[0]} rows for {n} sequences")
        return yc

    def decode_cache(self, n_samples):
        nbytes = V.lib().vqa_prior_decode_cache_bytes(n_samples, self.depth, self.context_length)
        return torch.empty(nbytes, dtype=torch.uint8, device=self.device)

    def sample(self, n_samples, max_length=None, x_cond=None, y_cond=None, return_attention_weights=False, seed=0,
               forced=None, return_logits=False):
        """autoregressive_fmha.py:162-240: (N, max_length + 1) int64 tokens starting with the start token, each
        next token = argmax(logits + Gumbel noise). One persistent decode launch."""
        L = self.context_length if max_length is None else int(max_length)
        if not 0 < L <= self.context_length:
            raise ValueError(f"max_length {L} outside (0, {self.context_length}]")
        xc = None
        if x_cond is not None:
            # autoregressive_fmha.py:145-148 asserts x_cond is [n_samples, max_length, d_model] before adding it:
            # the decode kernel reads x_cond[n, i] for every sample n and position i < L
            xc = self._cond(x_cond).float().contiguous()
            if xc.dim() != 3 or xc.shape[0] != n_samples or xc.shape[1] < L or xc.shape[2] != self.d_model:
                raise ValueError(f"x_cond shape {tuple(xc.shape)}: expected ({n_samples}, >= {L}, {self.d_model})")
            if xc.shape[1] != self.context_length:
                full = torch.zeros(n_samples, self.context_length, self.d_model, device=self.device)
                n = min(xc.shape[1], self.context_length)
                full[:, :n] = xc[:, :n]
                xc = full
        tokens = torch.empty(n_samples, L + 1, dtype=torch.int64, device=self.device)
        logits = (torch.empty(n_samples, L, self.bins, dtype=torch.float32, device=self.device)
                  if return_logits else None)
        if forced is not None:
            forced = torch.as_tensor(forced, device=self.device).long().contiguous()
            if tuple(forced.shape) != (n_samples, L + 1):
                raise ValueError(f"forced shape {tuple(forced.shape)}: expected ({n_samples}, {L + 1})")
        yc = self._ycond(y_cond, n_samples)
        layers = [ly.layer_desc() for ly in self.transformer.layers]
        ow, ob = self.store.view(self.out_kernel), self.store.view(self.out_bias)
        if self.bins % 4:
            # the decode kernel's head mat-vec takes 16-byte column chunks: zero-pad the vocabulary to a multiple
            # of 4 (the sampler's default 513 bins); the padded columns are never sampled
            ld = -(-self.bins // 4) * 4
            owp = torch.zeros(self.d_model, ld, device=self.device)
            owp[:, :self.bins] = ow
            obp = torch.zeros(ld, device=self.device)
            obp[:self.bins] = ob
            ow, ob = owp, obp
        V.prior_decode(layers, self.store.view(self.emb_name), self._pos().contiguous(), ow, ob, tokens,
                       self.decode_cache(n_samples), L, self.context_length, self.heads, self.blocks,
                       self.start_token, seed, ycond=yc, xcond=xc, forced=forced, logits=logits, bins=self.bins)
        if return_logits:
            return tokens, logits
        if return_attention_weights:
            return tokens, {}  # the decode kernel keeps no attention-weight tensors
        return tokens

    def sequence_loss(self, inputs, targets, x_cond=None, y_cond=None, loss_fn=None):
        """(N,) mean per-token cross entropy of `targets` under the model fed `inputs` (autoregressive.py:189-201
        per sequence). loss_fn: None for the fused head (logits never written), or a callable on
        (targets, (N, T, bins) logits) -> (N, T) losses (the logits are then materialised)."""
        inputs = torch.as_tensor(inputs, device=self.device).long().contiguous()
        targets = torch.as_tensor(targets, device=self.device).long().contiguous()
        N, T = inputs.shape
        if loss_fn is not None:
            logits, _ = self(inputs, x_cond=x_cond, y_cond=y_cond)
            return torch.as_tensor(loss_fn(targets, logits), device=self.device).float().reshape(N, T).mean(dim=1)
        # every factorization is causal in time, so a partial last block is padded to the block length (the
        # padded positions do not reach the first T) — the attention kernels take whole blocks
        l = self.context_length // self.blocks
        Tp = -(-T // l) * l
        if Tp != T:
            inputs = torch.nn.functional.pad(inputs, (0, Tp - T))
            targets = torch.nn.functional.pad(targets, (0, Tp - T))
        xc = self._cond(x_cond)
        if xc is not None and xc.shape[1] > Tp:
            xc = xc[:, :Tp].contiguous()
        with torch.no_grad():
            h = self.hidden(inputs, False, xc, self._ycond(y_cond))
            lse = torch.empty(N * Tp, dtype=torch.float32, device=self.device)
            loss_row = torch.empty_like(lse)
            V.head_fwd(h, self._wt(self.cdt), self.store.view(self.out_bias), lse, targets=targets, loss_row=loss_row)
        return loss_row.reshape(N, Tp)[:, :T].mean(dim=1)

    def random_sample(self, loss_fn=None, seq_length=None, iterations=10, batch_per_iter=4, token_freq=0.50, seed=0):
        """autoregressive_fmha.py:242-302 random search: `iterations` rounds of `batch_per_iter` ancestral samples
        (round i draws its Gumbel noise with seed + i); each sample is scored by its own mean token loss under the
        model, and a round's samples are taken in ascending loss while they beat the best so far — skipping any
        in which one token fills >= int(seq_length * token_freq) of the (start-token-led) sequence. Returns (best
        (seq_length + 1,) int64 sample with its start token — zeros (1, seq_length) if none qualified — , best
        loss)."""
        L = self.context_length if seq_length is None else int(seq_length)
        best_loss = 1e10
        best = torch.zeros(1, L, dtype=torch.int64, device=self.device)
        limit = int(L * token_freq)
        for i in range(iterations):
            out = self.sample(batch_per_iter, max_length=L, seed=seed + i)  # (N, L + 1), start token first
            loss = self.sequence_loss(out[:, :-1], out[:, 1:], loss_fn=loss_fn).cpu()
            for k in torch.argsort(loss, stable=True).tolist():
                cur = float(loss[k])
                if not cur < best_loss:
                    break
                cand = out[k]
                _, counts = torch.unique(cand, return_counts=True)
                if int(counts.max()) >= limit:
                    continue  # the reference prints "Token ... occurred ... Times! Skipping..."
                best_loss, best = cur, cand
        return best, best_loss

    @property
    def trainable_variables(self):
        return [self.store.view(n) for n, _, _ in self.store.specs if n.startswith(self.prefix + "/")]


class Prior:
    """prior.py:102-372: trains one level's FMHABasedAutoregressiveModel on the VQ-VAE's codes.

    train_step(x) takes raw audio (N, T, 1) (encoded with `vqvae_model`) or the codes themselves (N, T_l) int64.
    Returns {"loss", "perplexity(per word)", "accuracy"} running means (device tensors)."""

    def __init__(self, level, z_shapes, bins, down_depth, strides, vqvae_model, prior_kwargs, x_cond_kwargs,
                 prior_monitor=None, genre_classes=None, dtype="fp32", device="cuda", seed=1, learning_rate=1e-3,
                 process_group=None, **kwargs):
        assert len(down_depth) == len(strides) == len(z_shapes)
        self.level, self.z_shapes, self.levels = level, z_shapes, len(z_shapes)
        self.z_shape = z_shapes[level]
        self.context_length = int(np.prod(self.z_shape))
        self.bins, self.genre_bins = bins, genre_classes
        self.vqvae = vqvae_model
        self.device = torch.device(device)
        self.prior = FMHABasedAutoregressiveModel(
            target_vocab_size=bins, width=prior_kwargs["width"], depth=prior_kwargs["depth"],
            heads=prior_kwargs["heads"], blocks=prior_kwargs["blocks"], attn_stacks=prior_kwargs["attn_stacks"],
            drop_out_rate=prior_kwargs.get("drop_out_rate", 0.1), context_length=self.z_shape, zq_shapes=z_shapes,
            level=level, levels=self.levels, downs=down_depth, strides=strides, cond_kwargs=x_cond_kwargs,
            dtype=dtype, device=device, seed=seed, grad_extra=2, label_bins=genre_classes)
        # data parallel (one process per GPU): ONE all_reduce per step over [gradients | loss, accuracy]
        self.process_group = process_group
        st = self.prior.store
        self.bucket = st.grad
        self._scalars = self.bucket[st.size:st.size + 2]
        self.label_conditioner = None
        # prior.py:154-157 (LabelConditioner(genre_bins, width)): built into the prior's parameter store
        self.label_conditioner = self.prior.label_conditioner
        self.optimizer = Adam(learning_rate=learning_rate)
        self.optimizer.build(self.prior.store)  # its device step counter also drives dropout / teacher forcing
        self.train_loss_tracker = Mean("train_loss", self.device)
        self.train_accuracy_tracker = Mean("train_accuracy", self.device)
        self.train_monitor = prior_monitor
        self.teacher_seed = 3
        self._step = 0
        self._graph = None

    @property
    def metrics(self):
        return [self.train_loss_tracker, self.train_accuracy_tracker]

    def compile(self, optimizer=None, **kwargs):
        """keras Model.compile (the reference compiles with tf.keras.optimizers.Adam(), prior.py:436): a
        vqa_optim.Adam whose learning_rate is a float or a LearningRateSchedule such as
        schedules.CustomSchedule(d_model) (src/transformer/multi_head_attention.py:82-101), evaluated on the
        device each step. A captured step is dropped (it holds the previous optimizer's buffers)."""
        self.optimizer = optimizer or Adam()
        self.optimizer.build(self.prior.store)
        self._graph = None

    def reset_metrics(self):
        for m in self.metrics:
            m.reset_state()

    def set_train_monitor(self, train_monitor):
        self.train_monitor = train_monitor

    def get_cond(self, zs, start, end):
        """autoregressive_fmha.py:82-105."""
        if self.level == self.levels - 1:
            return None
        r = self.prior.cond_downsample_rate
        assert start % r == end % r == 0
        return zs[self.level + 1][:, start // r:end // r]

    def _codes(self, x):
        """-> (codes (N, T_l) int64, upper-level codes or None, labels (N,) int64 or None).

        x is raw audio (N, T, 1) (encoded with `vqvae_model`: this level's codes and, for the upsampler
        conditioning, the level above's, prior.py:257-260) or the codes themselves (int64). A tuple carries the
        extras: (audio, y) as the reference's train_step takes it (prior.py:251-254), (codes, upper_codes) for a
        prior conditioned on the level above, (codes, y) / (codes, upper_codes, y) with genre labels."""
        extras = []
        if isinstance(x, (tuple, list)):
            x, extras = x[0], list(x[1:])
        x = torch.as_tensor(x, device=self.device)
        conditioned = self.prior.conditioner is not None
        if x.dtype == torch.int64:
            codes, upper = x.contiguous(), None
            if conditioned:
                if not extras:
                    raise ValueError("a conditioned prior needs (codes, upper_level_codes)")
                upper = torch.as_tensor(extras.pop(0), device=self.device).long().contiguous()
        else:
            zs = self.vqvae.encode(x, start_level=self.level, end_level=self.levels)
            codes = zs[0].contiguous()
            upper = zs[1] if self.level != self.levels - 1 else None
        y = None
        if extras and extras[0] is not None:
            if self.label_conditioner is None:
                raise ValueError("labels given to a prior built without genre_classes")
            y = torch.as_tensor(extras[0], device=self.device).long().reshape(-1).contiguous()
            if y.numel() != codes.shape[0]:
                raise ValueError(f"{y.numel()} labels for {codes.shape[0]} sequences")
        return codes, upper, y

    def results(self):
        loss = self.train_loss_tracker.result()
        return {"loss": loss, "perplexity(per word)": torch.exp(loss), "accuracy": self.train_accuracy_tracker.result()}

    # -------------------------------------------------------------- the step
    def _world(self):
        return vqa_dp.world_size(self.process_group)

    def _label_embed(self, y):
        """LabelConditioner(y) (label_conditioners.py:26-45) as the (N, width) fp32 rows the embedding kernel puts at
        position 0."""
        if y is None:
            return None
        lc = self.label_conditioner
        out = torch.empty(y.numel(), self.prior.d_model, dtype=torch.float32, device=self.device)
        V.embedding_fwd(lc.store.view(lc.name), y, out)
        return out

    def _compute(self, codes, upper, teacher_force_rate, tf_mask=None, y=None):
        """Both teacher-forcing passes and the backward: gradients and [loss, accuracy] sums in the bucket."""
        m, st = self.prior, self.prior.store
        N, T = codes.shape
        M = N * T
        dev = self.device
        seed = self.teacher_seed
        ctr = self.optimizer.iterations
        row_offset = vqa_dp.rank(self.process_group) * M
        xc = m._cond(upper, save=True) if upper is not None else None
        yc = self._label_embed(y)
        m.prep_weights(bwd=True)
        # pass 1: teacher-forced input, argmax of the logits (prior.py:277-282)
        latent = torch.empty_like(codes)
        V.tf_mix(codes, None, None, latent, m.start_token)
        wt = m._wt(m.cdt)
        b = st.view(m.out_bias)
        with torch.no_grad():
            h0 = m.hidden(latent, True, xc, yc, seed=seed * 7919 + 1, counter=ctr, prepped=True, row0=row_offset)
            lse0 = torch.empty(M, dtype=torch.float32, device=dev)
            amax = torch.empty(N, T, dtype=torch.int64, device=dev)
            V.head_fwd(h0, wt, b, lse0, amax=amax)
            del h0
        # mix (prior.py:283-290) and pass 2 with gradients
        batch_input = torch.empty_like(codes)
        mask = None if tf_mask is None else torch.as_tensor(tf_mask, device=dev).to(torch.uint8).contiguous()
        V.tf_mix(codes, amax, mask, batch_input, m.start_token, rate=float(teacher_force_rate), seed=seed,
                 counter=ctr, row_offset=row_offset)
        h = m.hidden(batch_input, True, xc, yc, save=True, seed=seed * 7919 + 2, counter=ctr, prepped=True,
                     row0=row_offset)
        lse = torch.empty(M, dtype=torch.float32, device=dev)
        loss_row = torch.empty(M, dtype=torch.float32, device=dev)
        correct = torch.empty(M, dtype=torch.float32, device=dev)
        V.head_fwd(h, wt, b, lse, targets=codes, loss_row=loss_row, correct=correct)
        V.rowsum(loss_row, 1, M, 1.0 / M, self._scalars[0:1])
        V.rowsum(correct, 1, M, 1.0 / M, self._scalars[1:2])
        self._last_batch_input = batch_input
        deferred = V.Deferred()
        st.deferred = deferred
        post = []
        try:
            dh = torch.empty_like(h)
            V.head_bwd(h, wt, b, codes, lse, 1.0 / M, dh, st.grad_view(m.out_kernel), st.grad_view(m.out_bias),
                       deferred=deferred)
            for ly in reversed(m.transformer.layers):
                dh = ly.backward(dh, T, deferred, post)
            # embeddings: x0 = dropout(E[tok] * sqrt(d) + pos) (+ x_cond), position 0 = the label embedding
            # when labels are given (autoregressive_fmha.py:119-151)
            if xc is not None:
                m.conditioner.backward(dh)
            if m.rate > 0:  # the embedding dropout's mask, in place (dh is not read again)
                V.dropout_(dh, m.rate, seed * 7919 + 2, V.EMB_DROPOUT_SALT, ctr, elem_offset=row_offset * m.d_model)
            if m.use_pos_embedding:
                V.colsum(dh, st.grad_view(m.pos_name), N, T * m.d_model, T * m.d_model)
            gl = None
            if y is not None:
                lc = self.label_conditioner
                gl = st.grad_view(lc.name)
                gl.zero_()
                V.embedding_bwd(dh[:, 0, :].contiguous(), y, gl)
                dh[:, 0, :].zero_()  # the start token's row does not reach the token table
            gt = st.grad_view(m.emb_name)
            gt.zero_()
            V.embedding_bwd(dh, batch_input, gt)
            deferred.flush()
            V.scale_f32_(gt, math.sqrt(m.d_model))
            if gl is not None:
                V.scale_f32_(gl, math.sqrt(m.d_model))
            for dst, extra in post:
                V.axpy(dst, extra, dst)
        finally:
            st.deferred = None
        if m.use_pos_embedding and T < m.context_length:
            st.grad_view(m.pos_name)[T:].zero_()

    def _exchange(self):
        vqa_dp.exchange(self.bucket, self.process_group)

    def _apply(self):
        """Keras Adam on the (rank-mean) gradients, then the trackers on the global means."""
        w = self._world()
        self.optimizer.apply(self.prior.store, grad_scale=1.0 / w)
        self.train_loss_tracker.update_state(self._scalars[0] / w)
        self.train_accuracy_tracker.update_state(self._scalars[1] / w)

    def train_step(self, x, teacher_force_rate=0.2, tf_mask=None):
        """prior.py:241-335. tf_mask (N, T) bool overrides the random teacher-forcing draw (parity tests)."""
        codes, upper, y = self._codes(x)
        # the captured graph bakes in its teacher-forcing rate: another rate (e.g. a schedule) runs eagerly
        if (self._graph is not None and tf_mask is None and self._graph_fits(codes, upper, y)
                and float(teacher_force_rate) == self._graph_rate):
            self._graph_in[0].copy_(codes)
            if upper is not None:
                self._graph_in[1].copy_(upper)
            if y is not None:
                self._graph_in[2].copy_(y)
            g1, g2 = self._graph
            g1.replay()
            if g2 is not None:
                self._exchange()
                g2.replay()
            self._step += 1
            return self.results()
        self._compute(codes, upper, teacher_force_rate, tf_mask, y)
        self._exchange()
        self._apply()
        self._step += 1
        return self.results()

    def _graph_fits(self, codes, upper, y):
        c, u, l = self._graph_in
        same = lambda a, b: (a is None) == (b is None) and (a is None or a.shape == b.shape)
        return same(codes, c) and same(upper, u) and same(y, l)

    def test_step(self, x):
        """prior.py:337-372: loss / accuracy of the teacher-forced input (no mixing, no update). As in the
        reference, the batch's values go into train_loss_tracker / train_accuracy_tracker and the running means
        are returned (a keras evaluate loop over several batches reports their mean)."""
        m = self.prior
        codes, upper, y = self._codes(x)
        N, T = codes.shape
        M = N * T
        with torch.no_grad():
            latent = torch.empty_like(codes)
            V.tf_mix(codes, None, None, latent, m.start_token)
            h = m.hidden(latent, False, m._cond(upper), self._label_embed(y))
            lse = torch.empty(M, dtype=torch.float32, device=self.device)
            lr, cr = torch.empty_like(lse), torch.empty_like(lse)
            V.head_fwd(h, m._wt(m.cdt), m.store.view(m.out_bias), lse, targets=codes, loss_row=lr, correct=cr)
            out = torch.empty(2, dtype=torch.float32, device=self.device)
            V.rowsum(lr, 1, M, 1.0 / M, out[0:1])
            V.rowsum(cr, 1, M, 1.0 / M, out[1:2])
        self.train_loss_tracker.update_state(out[0])
        self.train_accuracy_tracker.update_state(out[1])
        return self.results()

    def evaluate(self, x=None, y=None, batch_size=None, verbose=0, steps=None, return_dict=False, **kwargs):
        """keras Model.evaluate over test_step (prior.py:337-372), as src/callback/monitors.py:81 calls it on the
        validation dataset: the loss / accuracy trackers reset, test_step per batch, their running means returned
        (vqa_module.keras_evaluate)."""
        return keras_evaluate(self, x, y, batch_size=batch_size, verbose=verbose, steps=steps,
                              return_dict=return_dict)

    def capture_train_step(self, codes_example, teacher_force_rate=0.2, warmup=1):
        """Record the whole step (both passes, the conditioner, backward, Adam, metrics) as one hipGraph — two
        around the eager all_reduce under data parallelism; later train_step calls with the same shapes copy the
        codes (upper-level codes, labels) in and replay (the teacher-forcing draw and dropout advance on the
        device)."""
        codes, upper, y = self._codes(codes_example)
        self._graph_in = tuple(None if t is None else t.clone() for t in (codes, upper, y))
        c, u, l = self._graph_in
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._compute(c, u, teacher_force_rate, None, l)
                self._exchange()
                self._apply()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        pool = torch.cuda.graph_pool_handle()
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1, pool=pool, capture_error_mode="thread_local"):
            self._compute(c, u, teacher_force_rate, None, l)
            if not vqa_dp.active(self.process_group):
                self._apply()
        g2 = None
        if vqa_dp.active(self.process_group):  # two graphs around the eager all_reduce
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, pool=pool, capture_error_mode="thread_local"):
                self._apply()
        self._graph = (g1, g2)
        self._graph_rate = float(teacher_force_rate)
        torch.cuda.synchronize(self.device)

    # -------------------------------------------------------------- checkpoint
    def save(self, path: str):
        """Checkpoint to disk (the reference's prior trains under the same injected checkpoint manager as the
        VQ-VAE, src/callback/monitors.py): tensors, ints and strings only — `torch.load(path, weights_only=True)`
        reads it. Weights (the ConditionerNet's and the genre table's included), Adam moments and step (the step
        also drives teacher forcing and dropout), and the loss / accuracy trackers: resuming reproduces the
        uninterrupted run bit for bit."""
        st = self.prior.store
        out = {"format": f"vqa-prior/{CKPT_VERSION}", "param_names": [n for n, _, _ in st.specs],
               "layout": st.layout_record(),
               "config": {"level": self.level, "bins": self.bins, "context_length": self.context_length,
                          "width": self.prior.d_model, "depth": self.prior.depth, "heads": self.prior.heads,
                          "blocks": self.prior.blocks, "genre_classes": self.genre_bins},
               "weights": st.flat.detach().cpu().clone(),
               "adam_m": self.optimizer.m.detach().cpu().clone(), "adam_v": self.optimizer.v.detach().cpu().clone(),
               "iterations": int(self.optimizer.iterations.item()), "step": int(self._step),
               "trackers": torch.stack([t._acc.detach().cpu() for t in self.metrics])}
        torch.save(out, path)

    def load(self, path: str):
        """Restore a `save` checkpoint (loaded weights-only: nothing in the file is executed); format /2 is
        copied tensor by tensor through its recorded layout, /1 in the layout its length identifies."""
        ck = torch.load(path, map_location="cpu", weights_only=True)
        st = self.prior.store
        lay = checkpoint_layout(ck, st, "prior", path)
        st.flat.copy_(st.from_layout(ck["weights"], lay, path).to(self.device))
        self.optimizer.m.copy_(st.from_layout(ck["adam_m"], lay, f"{path} (adam_m)").to(self.device))
        self.optimizer.v.copy_(st.from_layout(ck["adam_v"], lay, f"{path} (adam_v)").to(self.device))
        self.optimizer.iterations.fill_(int(ck["iterations"]))
        self._step = int(ck["step"])
        for t, acc in zip(self.metrics, ck["trackers"]):
            t._acc.copy_(acc.to(self.device))

    def sample(self, n_samples, z_cond=None, y=None, return_attn_weights=False, seed=0):
        """prior.py:374-408: one window of n_ctx tokens, the start token first (as FMHABasedAutoregressiveModel.sample
        returns it; VQVAESampler drops it). y: genre labels (N,) through the LabelConditioner."""
        if z_cond is not None and int(z_cond.shape[0]) != n_samples:
            raise ValueError(f"Batch Size not matching, Expected:{n_samples}, Getting: {int(z_cond.shape[0])}")
        y_cond = None
        if y is not None:
            if self.label_conditioner is None:
                raise ValueError("labels given to a prior built without genre_classes")
            y = torch.as_tensor(y, device=self.device).long().reshape(-1).contiguous()
            if y.numel() != n_samples:
                raise ValueError(f"Batch Size not matching, Expected:{n_samples}, Getting: {y.numel()}")
            y_cond = self._label_embed(y)
        return self.prior.sample(n_samples, x_cond=z_cond, y_cond=y_cond, seed=seed,
                                 return_attention_weights=return_attn_weights)
