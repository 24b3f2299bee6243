"""Upper-level conditioner — drop-in for the reference src/conditioner/conditioners.py (ConditionerNet).

conditioners.py:9-72   ConditionerNet(cond_shape, bins, embed_width, residual_width, residual_depth, down_depth,
                       stride, dilation_factor=1, reverse_dilation=False, dilation_cycle=None):
                       keras.Sequential([Embedding(bins, embed_width),
                                         DecoderConvBlock(embed_width, residual_width, residual_depth, stride=stride,
                                                          dilation_factor, reverse_dilation, down_depth, dilation_cycle),
                                         LayerNormalization(axis=-1, epsilon=1e-6)])
conditioners.py:74-91  call: asserts the input length == cond_shape[0] and the output length ==
                       cond_shape[0] * stride ** down_depth.
The prior builds it with embed_width = d_model (128), residual_width 32, residual_depth 8, dilation_factor 3,
dilation_cycle 4 (Sampler.py:25, prior.py:415; autoregressive_fmha.py:57-60): upper-level codes -> a
(B, L * stride^down_depth, 128) conditioning sequence for the level below.

MI355X path: the Embedding gather and LayerNorm are libvqa kernels (vqa_cond.hip); the DecoderConvBlock is the
VQ-VAE decoder's own conv / fused residual-block kernels (the 32-channel blocks with the cyclic dilations
1, 3, 9, 27, 1, 3, 9, 27 run on vqa_resblock). Backward is explicit (forward(save=True) then backward(dy)): the
LayerNorm and weight gradients are deterministic, the Embedding gradient is the fixed-order segment sum of
vqa_embedding_bwd.
"""
from __future__ import annotations

from typing import Optional

import torch

import vqa_lib as V
from encdec import DecoderConvBlock
from vqa_layers import ParamStore
from vqa_module import Layer


class ConditionerNet(Layer):
    def __init__(self, cond_shape, bins, embed_width, residual_width, residual_depth, down_depth, stride,
                 dilation_factor=1, reverse_dilation=False, dilation_cycle=None, **kwargs):
        super().__init__(**kwargs)
        self.x_shape = tuple(cond_shape)
        self.bins = bins
        self.depth = self.down_depth = down_depth
        self.width = self.embed_width = embed_width
        self.stride = stride
        self.epsilon = 1e-6
        self.block = DecoderConvBlock(embed_width, residual_width, residual_depth, stride=stride,
                                      dilation_factor=dilation_factor, reverse_dilation=reverse_dilation,
                                      down_depth=down_depth, dilation_cycle=dilation_cycle)
        self._saved = None

    def _build(self, store, prefix, input_dim=None):
        self.prefix = prefix
        self.table_name = store.add(f"{prefix}/embedding/embeddings", (self.bins, self.width), "uniform")
        self.block.build(store, f"{prefix}/block", self.width, self.cdt)
        self.gamma_name = store.add(f"{prefix}/layer_norm/gamma", (self.width,), "ones")
        self.beta_name = store.add(f"{prefix}/layer_norm/beta", (self.width,), "zeros")
        return self.width

    def _param_names(self):
        return [n for n, _, _ in self.store.specs if n.startswith(self.prefix + "/")]

    def build_standalone(self, device="cuda", dtype=torch.float32, seed=1):
        store = ParamStore()
        self.build(store, self.name, self.width, dtype)
        store.materialize(torch.device(device), seed=seed)
        return self

    def out_len(self) -> int:
        return self.x_shape[0] * self.stride ** self.down_depth

    def forward(self, idx: torch.Tensor, save: bool = False) -> torch.Tensor:
        """(N, L) int64 codes -> (N, L * stride^down_depth, embed_width) in the compute dtype."""
        N, L = idx.shape
        if L != self.x_shape[0]:  # conditioners.py:76-79
            raise ValueError(f"Upper Level Shape Not match: {L} != {self.x_shape[0]}")
        st = self.store
        e = torch.empty(N, L, self.width, dtype=self.cdt, device=idx.device)
        V.embedding_fwd(st.view(self.table_name), idx, e)
        h = self.block.forward(e, save)
        if h.shape[1] != self.out_len():  # conditioners.py:85-89
            raise ValueError(f"Upsampled Shape Not match: {h.shape[1]} != {self.out_len()}")
        y = torch.empty_like(h)
        V.layernorm_fwd(h, st.view(self.gamma_name), st.view(self.beta_name), y, self.epsilon)
        self._saved = (idx, h) if save else None
        return y

    def backward(self, dy: torch.Tensor):
        """Gradients of every parameter (written into the store's gradient buffer) from dL/dy."""
        idx, h = self._saved
        self._saved = None
        st = self.store
        dh = torch.empty_like(h)
        V.layernorm_bwd(h, dy.to(h.dtype).contiguous(), st.view(self.gamma_name), dh, st.grad_view(self.gamma_name),
                        st.grad_view(self.beta_name), self.epsilon, st.deferred)
        de = self.block.backward(dh)
        gt = st.grad_view(self.table_name)
        gt.zero_()
        V.embedding_bwd(de, idx, gt)

    def __call__(self, inputs, training: bool = False, **kwargs) -> torch.Tensor:
        dev = self.store.flat.device if self.built else torch.device("cuda")
        idx = torch.as_tensor(inputs).to(device=dev, dtype=torch.int64).contiguous()
        if not self.built:
            self.build_standalone(dev)
        with torch.no_grad():
            return self.forward(idx)

    call = __call__
