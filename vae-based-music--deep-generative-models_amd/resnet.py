"""Dilated residual stacks — drop-in for the reference resnet.py (ResnetConv1DBlock, DilatedResnet1D).

resnet.py:7-29   ResnetConv1DBlock: y = x + Conv1D_k3,d1(ReLU(Conv1D_k3,dil(ReLU(x))))
resnet.py:40-59  DilatedResnet1D: `depth` blocks, dilation dilation_factor**d (or **(d % dilation_cycle)),
                 reversed for decoders.
For 32 channels the whole block is ONE forward kernel (h kept on chip) and ONE backward kernel (h recomputed
from x; dx and all four weight gradients from one pass over dy and x) — csrc/vqa_resblock.hip. Other widths
run the two convs on the gather-conv kernels (ReLUs fused into the LDS staging, the residual add into the
epilogue, each conv's backward one kernel).
"""
from __future__ import annotations

from typing import List, Optional

import torch

import vqa_lib as V
from vqa_layers import Conv1D
from vqa_module import Layer


class ResnetConv1DBlock(Layer):
    def __init__(self, input_dim, filters, dilation=1, **kwargs):
        super().__init__(**kwargs)
        self.input_dim, self.filters, self.dilation = input_dim, filters, dilation
        self._saved = None
        self._fused = None

    def _build(self, store, prefix, input_dim):
        assert input_dim == self.input_dim, f"{prefix}: input_dim {input_dim} != {self.input_dim}"
        self.conv_a = Conv1D(store, f"{prefix}/conv_a", self.input_dim, self.filters, 3, 1, self.dilation)
        self.conv_b = Conv1D(store, f"{prefix}/conv_b", self.filters, self.input_dim, 3, 1, 1)
        return self.input_dim

    def fused(self) -> bool:
        """The whole block runs as one forward and one backward kernel (vqa_resblock_*) when supported."""
        if self._fused is None:
            self._fused = (self.input_dim == self.filters and
                           V.resblock_supported(self.input_dim, self.dilation, V.dtype_code(self.cdt)))
        return self._fused

    def forward(self, x, save=False):
        if self.fused() and x.dtype == self.cdt:
            # h stays on chip; the backward recomputes it from x, so only x is saved
            y = torch.empty_like(x)
            V.resblock_fwd(x, self.conv_a.w, self.conv_a.b, self.conv_b.w, self.conv_b.b, y, self.dilation)
            self._saved = (x, None) if save else None
            return y
        h = self.conv_a.forward(x, self.cdt, pre_relu=True)
        y = self.conv_b.forward(h, self.cdt, pre_relu=True, residual=x)
        self._saved = (x, h) if save else None
        return y

    def backward(self, dy):
        x, h = self._saved
        self._saved = None
        if h is None:
            st = self.store
            dx = torch.empty_like(x)
            V.resblock_bwd(dy, x, self.conv_a.w, self.conv_a.b, self.conv_b.w, self.conv_b.b, dx,
                           st.grad_view(f"{self.conv_a.name}/kernel"), st.grad_view(f"{self.conv_a.name}/bias"),
                           st.grad_view(f"{self.conv_b.name}/kernel"), st.grad_view(f"{self.conv_b.name}/bias"),
                           self.dilation, st.deferred)
            return dx
        # each conv's data- and weight-gradient in one kernel: its input (h, x) is both the ReLU' mask and
        # the weight-gradient operand, so it is read once
        dh = self.conv_b.backward_data_weight(dy, h, self.cdt, pre_relu=True)
        return self.conv_a.backward_data_weight(dh, x, self.cdt, pre_relu=True, residual=dy)


class DilatedResnet1D(Layer):
    def __init__(self, input_dim, depth, dilation_factor=1, reverse_dilation=False, dilation_cycle=None, **kwargs):
        super().__init__(**kwargs)
        self.input_dim, self.depth = input_dim, depth

        def _get_dilation(d):  # resnet.py:44-48
            return dilation_factor ** d if dilation_cycle is None else dilation_factor ** (d % dilation_cycle)

        self.dilations: List[int] = [_get_dilation(d) for d in range(depth)]
        if reverse_dilation:  # resnet.py:54-55
            self.dilations = self.dilations[::-1]
        self.blocks = [ResnetConv1DBlock(input_dim, input_dim, dilation=d) for d in self.dilations]

    def _build(self, store, prefix, input_dim):
        for j, blk in enumerate(self.blocks):
            blk.build(store, f"{prefix}/rb{j}", input_dim, self.cdt)
        return input_dim

    def forward(self, x, save=False):
        for blk in self.blocks:
            x = blk.forward(x, save)
        return x

    def backward(self, dy):
        for blk in reversed(self.blocks):
            dy = blk.backward(dy)
        return dy
