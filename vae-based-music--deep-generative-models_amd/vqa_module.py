"""Keras-like layer base: deferred build, standalone __call__, explicit forward/backward.

A layer registers its weights in a ParamStore at build() (the input channel count is known then, as
in Keras' deferred build). Used standalone, `layer(x)` builds a private store on first call with the
Keras default initialisers and runs the forward on the GPU. Inside VQVAE every layer shares the model's
store so the whole model's weights / gradients are two flat buffers.
"""
from __future__ import annotations

from typing import Optional

import torch

from vqa_layers import ParamStore


class Layer:
    def __init__(self, name: Optional[str] = None, **kwargs):
        self.name = name or type(self).__name__
        self.built = False
        self.cdt = torch.float32
        self.store: Optional[ParamStore] = None

    # subclasses implement _build(store, prefix, input_dim) -> output_dim, forward, backward
    def build(self, store: ParamStore, prefix: str, input_dim: int, cdt: torch.dtype) -> int:
        self.store, self.cdt = store, cdt
        out = self._build(store, prefix, input_dim)
        self.built = True
        return out

    def _standalone_build(self, x: torch.Tensor, seed: int = 1):
        store = ParamStore()
        cdt = x.dtype if x.dtype in (torch.float32, torch.bfloat16) else torch.float32
        self.build(store, self.name, x.shape[-1], cdt)
        store.materialize(x.device, seed=seed)

    def __call__(self, x: torch.Tensor, training: bool = False, **kwargs) -> torch.Tensor:
        if not self.built:
            self._standalone_build(x)
        return self.forward(x, save=False)

    def forward(self, x, save=False):
        raise NotImplementedError

    def backward(self, dy):
        raise NotImplementedError

    @property
    def weights(self):
        return {n: self.store.view(n) for n in self._param_names()} if self.store else {}

    def _param_names(self):
        return []
