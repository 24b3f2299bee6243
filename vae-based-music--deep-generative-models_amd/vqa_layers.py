"""Parameter store and the two convolution primitives (keras Conv1D / Conv1DTranspose, padding='same').

All trainable fp32 weights of a model live in ONE flat device buffer, their gradients in one flat
buffer (the head of the data-parallel all-reduce bucket) — so Adam is one launch and the gradient
exchange is one RCCL call. Activations are channels-last (B, T, C) in the model's compute dtype
(bf16 or fp32); the waveform ends (1 channel) are fp32.

Each primitive has forward / backward_data / backward_weight that call the C-ABI (vqa_lib). Layers
built on them save what their backward needs during forward; nothing is recomputed.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

import vqa_lib as V


class ParamStore:
    """Flat fp32 parameter / gradient storage with named views (Keras kernel layouts). Every tensor starts on a
    16-byte boundary (offsets are multiples of 4 floats; the gaps stay zero, in the weights and the gradients),
    so the kernels' 16-byte weight loads stay aligned whatever the sizes before it (a 513-bin head bias, a
    1-channel output conv's bias)."""

    ALIGN = 4  # floats

    def __init__(self):
        self.specs: List[Tuple[str, Tuple[int, ...], str]] = []  # (name, shape, init)
        self.offsets: Dict[str, Tuple[int, Tuple[int, ...]]] = {}
        self.size = 0   # buffer length in floats (with the alignment gaps)
        self.count = 0  # trainable values
        self.flat: Optional[torch.Tensor] = None
        self.grad: Optional[torch.Tensor] = None
        self.deferred = None  # a vqa_lib.Deferred while a model step batches its weight-gradient reductions

    def add(self, name: str, shape: Tuple[int, ...], init: str) -> str:
        if name in self.offsets:
            raise ValueError(f"duplicate parameter {name}")
        n = int(np.prod(shape))
        off = -(-self.size // self.ALIGN) * self.ALIGN
        self.offsets[name] = (off, tuple(shape))
        self.specs.append((name, tuple(shape), init))
        self.size = off + n
        self.count += n
        return name

    def init_values(self, seed: int = 1) -> Dict[str, np.ndarray]:
        """keras defaults (numpy, registration order): glorot_uniform conv kernels, zero biases; Embedding
        'uniform' = U(-0.05, 0.05); LayerNormalization gamma 'ones', beta zeros."""
        rng = np.random.default_rng(seed)
        vals = {}
        for name, shape, init in self.specs:
            if init == "glorot_uniform":
                if len(shape) == 2:  # Dense kernel (in, out)
                    lim = math.sqrt(6.0 / (shape[0] + shape[1]))
                else:  # keras fans of an N-D kernel: receptive field prod(shape[:-2])
                    rf = int(np.prod(shape[:-2]))
                    lim = math.sqrt(6.0 / (rf * shape[-2] + rf * shape[-1]))
                vals[name] = rng.uniform(-lim, lim, size=shape).astype(np.float32)
            elif init == "uniform":
                vals[name] = rng.uniform(-0.05, 0.05, size=shape).astype(np.float32)
            elif init == "ones":
                vals[name] = np.ones(shape, np.float32)
            else:
                vals[name] = np.zeros(shape, np.float32)
        return vals

    def materialize(self, device, grad_buffer: Optional[torch.Tensor] = None, seed: int = 1):
        self.flat = torch.empty(self.size, dtype=torch.float32, device=device)
        self.grad = grad_buffer if grad_buffer is not None else torch.zeros(self.size, dtype=torch.float32,
                                                                            device=device)
        assert self.grad.numel() >= self.size
        self.set_values(self.init_values(seed))

    def view(self, name: str) -> torch.Tensor:
        off, shape = self.offsets[name]
        return self.flat[off:off + int(np.prod(shape))].view(shape)

    def grad_view(self, name: str) -> torch.Tensor:
        off, shape = self.offsets[name]
        return self.grad[off:off + int(np.prod(shape))].view(shape)

    def set_values(self, vals: Dict[str, np.ndarray]):
        host = np.zeros(self.size, np.float32)
        cur = self.flat.detach().cpu().numpy() if self.flat is not None else None
        for name, (off, shape) in self.offsets.items():
            n = int(np.prod(shape))
            if name in vals:
                v = np.asarray(vals[name], np.float32)
                if v.shape != shape:
                    raise ValueError(f"{name}: shape {v.shape} != {shape}")
                host[off:off + n] = v.reshape(-1)
            elif cur is not None:
                host[off:off + n] = cur[off:off + n]
            else:
                raise KeyError(f"missing value for {name}")
        self.flat.copy_(torch.from_numpy(host))

    def values(self) -> Dict[str, np.ndarray]:
        host = self.flat.detach().cpu().numpy()
        return {n: host[o:o + int(np.prod(s))].reshape(s).copy() for n, (o, s) in self.offsets.items()}

    def grads(self) -> Dict[str, np.ndarray]:
        host = self.grad[:self.size].detach().cpu().numpy()
        return {n: host[o:o + int(np.prod(s))].reshape(s).copy() for n, (o, s) in self.offsets.items()}

    # ---- checkpoint layout (format /2 saves it; /1 files are read by their length)
    def layout_record(self) -> Dict[str, List[int]]:
        """name -> [offset, *shape] of the flat buffers (weights, Adam m and v share it)."""
        return {n: [int(o), *map(int, s)] for n, (o, s) in self.offsets.items()}

    def legacy_layout(self, flat_len: int, what: str) -> Dict[str, List[int]]:
        """The layout a format-/1 checkpoint of this model was written in, told apart by its length: the
        16-byte-aligned layout (`size` floats) or the packed one of the first releases (`count` floats, every
        tensor right after the previous one). Anything else is rejected."""
        if flat_len == self.size:
            return self.layout_record()
        if flat_len == self.count:
            out, off = {}, 0
            for n, shape, _ in self.specs:
                out[n] = [off, *shape]
                off += int(np.prod(shape))
            return out
        raise ValueError(f"{what}: a flat buffer of {flat_len} floats fits neither this model's aligned layout "
                         f"({self.size}) nor its packed layout ({self.count})")

    def from_layout(self, flat: torch.Tensor, layout: Dict[str, List[int]], what: str) -> torch.Tensor:
        """Copy a saved flat buffer, tensor by tensor, into this store's layout (gaps zero) -> CPU fp32."""
        if set(layout) != set(self.offsets):
            raise ValueError(f"{what}: parameter names differ from this model's")
        flat = flat.detach().to("cpu", torch.float32).reshape(-1)
        out = torch.zeros(self.size, dtype=torch.float32)
        for n, (off, shape) in self.offsets.items():
            rec = layout[n]
            if tuple(rec[1:]) != tuple(shape):
                raise ValueError(f"{what}: {n} has shape {tuple(rec[1:])}, this model {tuple(shape)}")
            k = int(np.prod(shape))
            if rec[0] < 0 or rec[0] + k > flat.numel():
                raise ValueError(f"{what}: {n} lies outside the saved buffer")
            out[off:off + k] = flat[rec[0]:rec[0] + k]
        return out


CKPT_VERSION = 2


def checkpoint_layout(ck: dict, store: ParamStore, family: str, path: str) -> Dict[str, List[int]]:
    """The saved layout of a 'vqa-<family>/1' or '/2' checkpoint (see ParamStore.legacy_layout)."""
    fmt = ck.get("format")
    if fmt == f"vqa-{family}/{CKPT_VERSION}":
        return {n: list(v) for n, v in ck["layout"].items()}
    if fmt == f"vqa-{family}/1":
        if ck["param_names"] != [n for n, _, _ in store.specs]:
            raise ValueError(f"{path}: parameter layout differs from this model's")
        return store.legacy_layout(int(ck["weights"].numel()), path)
    raise ValueError(f"{path}: not a vqa-{family}/1 or /{CKPT_VERSION} checkpoint (format {fmt!r})")


def _flags_for(x: torch.Tensor, y_dtype: torch.dtype, cdt: torch.dtype) -> int:
    f = 0
    if cdt != torch.float32:
        if x.dtype == torch.float32:
            f |= V.X_F32
        if y_dtype == torch.float32:
            f |= V.Y_F32
    return f


class Conv1D:
    """keras layers.Conv1D(filters, kernel_size, strides, dilation_rate, padding='same') — kernel
    (K, C_in, C_out), bias (C_out). Replaces the TF conv at resnet.py:13,17, encdec.py:33,38,60,148."""

    def __init__(self, store: ParamStore, name: str, in_channels: int, filters: int, kernel_size: int,
                 strides: int = 1, dilation_rate: int = 1):
        self.store, self.name = store, name
        self.cin, self.cout, self.K, self.s, self.d = in_channels, filters, kernel_size, strides, dilation_rate
        store.add(f"{name}/kernel", (kernel_size, in_channels, filters), "glorot_uniform")
        store.add(f"{name}/bias", (filters,), "zeros")

    @property
    def w(self):
        return self.store.view(f"{self.name}/kernel")

    @property
    def b(self):
        return self.store.view(f"{self.name}/bias")

    def out_len(self, T: int) -> int:
        return -(-T // self.s)

    def pad(self, T: int) -> int:
        out = -(-T // self.s)
        return max((out - 1) * self.s + (self.K - 1) * self.d + 1 - T, 0) // 2

    def forward(self, x, cdt, pre_relu=False, residual=None, out_dtype=None):
        B, T, C = x.shape
        assert C == self.cin, f"{self.name}: expected {self.cin} channels, got {C}"
        To = self.out_len(T)
        ydt = out_dtype or cdt
        y = torch.empty((B, To, self.cout), dtype=ydt, device=x.device)
        fl = _flags_for(x, ydt, cdt) | (V.PRE_RELU if pre_relu else 0) | (V.ADD_RESIDUAL if residual is not None else 0)
        V.conv1d_fwd(x, self.w, self.b, residual, y, B, T, To, self.cin, self.cout, self.K, self.s, self.d,
                     self.pad(T), fl, V.dtype_code(cdt))
        return y

    def backward_data(self, dy, T_in, cdt, mask=None, residual=None, out_dtype=None):
        B, To, _ = dy.shape
        xdt = out_dtype or cdt
        dx = torch.empty((B, T_in, self.cin), dtype=xdt, device=dy.device)
        fl = _flags_for(dx, dy.dtype, cdt) | (V.POST_MASK if mask is not None else 0) | \
            (V.ADD_RESIDUAL if residual is not None else 0)
        V.conv1d_bwd_data(dy, self.w, mask, residual, dx, B, T_in, To, self.cin, self.cout, self.K, self.s, self.d,
                          self.pad(T_in), fl, V.dtype_code(cdt))
        return dx

    def backward_weight(self, x, dy, cdt, pre_relu=False):
        B, T, _ = x.shape
        fl = _flags_for(x, dy.dtype, cdt) | (V.PRE_RELU if pre_relu else 0)
        args = (x, dy, self.store.grad_view(f"{self.name}/kernel"), self.store.grad_view(f"{self.name}/bias"), B, T,
                dy.shape[1], self.cin, self.cout, self.K, self.s, self.d, self.pad(T), fl, V.dtype_code(cdt))
        if self.store.deferred is not None:
            V.conv1d_bwd_weight_deferred(*args, self.store.deferred)
        else:
            V.conv1d_bwd_weight(*args)


    def backward_data_weight(self, dy, x, cdt, pre_relu=False, residual=None):
        """backward_data (ReLU' mask = the conv input x when pre_relu) and backward_weight in one pass."""
        B, T, _ = x.shape
        dx = torch.empty((B, T, self.cin), dtype=cdt, device=dy.device)
        fl = _flags_for(x, dy.dtype, cdt) | (V.PRE_RELU if pre_relu else 0) | \
            (V.ADD_RESIDUAL if residual is not None else 0)
        V.conv1d_bwd_data_weight(dy, self.w, x, residual, dx, self.store.grad_view(f"{self.name}/kernel"),
                                 self.store.grad_view(f"{self.name}/bias"), B, T, dy.shape[1], self.cin, self.cout,
                                 self.K, self.s, self.d, self.pad(T), fl, V.dtype_code(cdt), self.store.deferred)
        return dx


class Conv1DTranspose:
    """keras layers.Conv1DTranspose(filters, 2*stride, strides=stride, padding='same') — kernel
    (K, C_out, C_in), bias (C_out). Replaces the TF op at encdec.py:67-68."""

    def __init__(self, store: ParamStore, name: str, in_channels: int, filters: int, kernel_size: int,
                 strides: int):
        self.store, self.name = store, name
        self.cin, self.cout, self.K, self.s = in_channels, filters, kernel_size, strides
        store.add(f"{name}/kernel", (kernel_size, filters, in_channels), "glorot_uniform")
        store.add(f"{name}/bias", (filters,), "zeros")

    @property
    def w(self):
        return self.store.view(f"{self.name}/kernel")

    @property
    def b(self):
        return self.store.view(f"{self.name}/bias")

    def pad(self, T_out: int) -> int:
        out = -(-T_out // self.s)
        return max((out - 1) * self.s + self.K - T_out, 0) // 2

    def forward(self, x, cdt, out_dtype=None):
        B, T, C = x.shape
        assert C == self.cin
        To = self.s * T
        ydt = out_dtype or cdt
        y = torch.empty((B, To, self.cout), dtype=ydt, device=x.device)
        V.conv1d_transpose_fwd(x, self.w, self.b, None, y, B, T, To, self.cin, self.cout, self.K, self.s,
                               self.pad(To), _flags_for(x, ydt, cdt), V.dtype_code(cdt))
        return y

    def backward_data(self, dy, cdt, mask=None, residual=None):
        B, To, _ = dy.shape
        T = To // self.s
        dx = torch.empty((B, T, self.cin), dtype=cdt, device=dy.device)
        fl = (V.POST_MASK if mask is not None else 0) | (V.ADD_RESIDUAL if residual is not None else 0)
        V.conv1d_transpose_bwd_data(dy, self.w, mask, residual, dx, B, T, To, self.cin, self.cout, self.K, self.s,
                                    self.pad(To), fl, V.dtype_code(cdt))
        return dx

    def backward_weight(self, x, dy, cdt):
        B, T, _ = x.shape
        args = (x, dy, self.store.grad_view(f"{self.name}/kernel"), self.store.grad_view(f"{self.name}/bias"), B, T,
                dy.shape[1], self.cin, self.cout, self.K, self.s, self.pad(dy.shape[1]), 0, V.dtype_code(cdt))
        if self.store.deferred is not None:
            V.conv1d_transpose_bwd_weight_deferred(*args, self.store.deferred)
        else:
            V.conv1d_transpose_bwd_weight(*args)
