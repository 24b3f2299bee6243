"""ctypes binding of libvqa.so (the C-ABI in include/vqa.h).

There is no CPU or PyTorch fallback: if libvqa.so is missing, `lib()` raises ImportError, and every op
raises VQAError with the library's own message when a call fails. Tensors are passed as raw device
pointers on torch's current HIP stream (so the calls are captured by torch.cuda.graph).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
# VQA_LIB_PATH: another build of the same sources (A/B and diagnosis tools only; the product loads libvqa.so)
LIB_PATH = os.environ.get("VQA_LIB_PATH") or os.path.join(HERE, "libvqa.so")

F32, BF16 = 0, 1
PRE_RELU, ADD_RESIDUAL, POST_MASK, X_F32, Y_F32 = 1, 2, 4, 8, 16

ABI_VERSION = 2  # include/vqa.h VQA_ABI_VERSION this binding is written against

EXPORTED = [
    "vqa_get_last_error", "vqa_version", "vqa_abi_version", "vqa_same_pad_left", "vqa_same_out_len",
    "vqa_conv1d_fwd", "vqa_conv1d_bwd_data", "vqa_conv1d_bwd_weight", "vqa_conv1d_bwd_weight_workspace",
    "vqa_conv1d_transpose_fwd", "vqa_conv1d_transpose_bwd_data", "vqa_conv1d_transpose_bwd_weight",
    "vqa_conv1d_transpose_bwd_weight_workspace",
    "vqa_vq_sqnorm", "vqa_vq_argmin", "vqa_vq_quantize", "vqa_vq_quantize_workspace", "vqa_vq_backward",
    "vqa_vq_reset_rows", "vqa_vq_ema_apply", "vqa_vq_ema_apply_derived", "vqa_reset_perm_index",
    "vqa_mse_loss", "vqa_mse_loss_workspace", "vqa_adam_keras", "vqa_lr_schedule", "vqa_counter_add",
    "vqa_conv1d_bwd_weight_partials", "vqa_conv1d_transpose_bwd_weight_partials", "vqa_reduce_partials",
    "vqa_conv1d_bwd_data_weight", "vqa_conv1d_bwd_data_weight_workspace",
    "vqa_spectral_loss", "vqa_spectral_loss_workspace", "vqa_stft_magnitude",
    "vqa_vq_argmin_split", "vqa_vq_split_bf16x3",
    "vqa_resblock_supported", "vqa_resblock_fwd", "vqa_resblock_bwd", "vqa_resblock_bwd_workspace",
    "vqa_spectral_target_workspace", "vqa_spectral_target", "vqa_spectral_loss_target_workspace",
    "vqa_spectral_loss_target", "vqa_dtail_supported", "vqa_dtail_workspace", "vqa_dtail_fwd", "vqa_dtail_bwd",
    "vqa_step_metrics", "vqa_synthetic_batch",
    "vqa_embedding_fwd", "vqa_embedding_bwd", "vqa_embedding_bwd_workspace", "vqa_layernorm_fwd",
    "vqa_layernorm_bwd", "vqa_layernorm_bwd_workspace",
    "vqa_seqlin_fwd", "vqa_seqlin_prep", "vqa_seqlin_fwd_prepped", "vqa_seqlin_fwd_ln_prepped", "vqa_seqlin_wgrad_workspace", "vqa_seqlin_wgrad", "vqa_prior_embed_fwd", "vqa_colsum",
    "vqa_axpy", "vqa_dropout", "vqa_scale_f32", "vqa_tf_mix", "vqa_attn_fwd", "vqa_attn_bwd", "vqa_head_wt",
    "vqa_head_fwd", "vqa_head_bwd_workspace", "vqa_head_bwd", "vqa_rowsum_workspace", "vqa_rowsum", "vqa_prior_decode_cache_bytes",
    "vqa_prior_decode",
]


class VQAError(RuntimeError):
    pass


class PartialsDesc(ctypes.Structure):
    """vqa_partials_desc (include/vqa.h)."""
    _fields_ = [("partials", ctypes.c_void_p), ("dw", ctypes.c_void_p), ("db", ctypes.c_void_p),
                ("nparts", ctypes.c_int), ("n", ctypes.c_int), ("n_w", ctypes.c_int), ("reserved", ctypes.c_int)]


_P, _I, _L, _S, _F, _U = (ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t, ctypes.c_float,
                          ctypes.c_uint64)
_CONV = [_I] * 11  # B T_in T_out C_in C_out K stride dilation pad flags dtype
_CONVT = [_I] * 10  # B T_in T_out C_in C_out K stride pad flags dtype

_SIGS = {
    "vqa_get_last_error": (ctypes.c_char_p, []),
    "vqa_version": (ctypes.c_char_p, []),
    "vqa_abi_version": (_I, []),
    "vqa_same_pad_left": (_I, [_I, _I, _I, _I]),
    "vqa_same_out_len": (_I, [_I, _I]),
    "vqa_conv1d_fwd": (_I, [_P, _P, _P, _P, _P] + _CONV + [_P]),
    "vqa_conv1d_bwd_data": (_I, [_P, _P, _P, _P, _P] + _CONV + [_P]),
    "vqa_conv1d_bwd_weight": (_I, [_P, _P, _P, _P] + _CONV + [_P, _S, _P]),
    "vqa_conv1d_bwd_weight_workspace": (_S, _CONV),
    "vqa_conv1d_transpose_fwd": (_I, [_P, _P, _P, _P, _P] + _CONVT + [_P]),
    "vqa_conv1d_transpose_bwd_data": (_I, [_P, _P, _P, _P, _P] + _CONVT + [_P]),
    "vqa_conv1d_transpose_bwd_weight": (_I, [_P, _P, _P, _P] + _CONVT + [_P, _S, _P]),
    "vqa_conv1d_transpose_bwd_weight_workspace": (_S, _CONVT),
    "vqa_vq_sqnorm": (_I, [_P, _P, _I, _I, _P]),
    "vqa_vq_argmin": (_I, [_P, _P, _P, _P, _P, _L, _I, _I, _I, _P]),
    "vqa_vq_quantize": (_I, [_P, _P, _P, _P, _P, _P, _P, _L, _I, _I, _F, _I, _P, _S, _P]),
    "vqa_vq_quantize_workspace": (_S, [_L, _I, _I, _I]),
    "vqa_vq_backward": (_I, [_P, _P, _P, _P, _P, _F, _L, _I, _I, _P]),
    "vqa_vq_reset_rows": (_I, [_P, _P, _L, _L, _L, _I, _I, _U, _P, _I, _I, _P]),
    "vqa_vq_ema_apply": (_I, [_P, _P, _P, _P, _P, _P, _P, _F, _F, _F, _P, _P, _I, _I, _P]),
    "vqa_vq_ema_apply_derived": (_I, [_P, _P, _P, _P, _P, _P, _P, _F, _F, _F, _P, _P, _P, _P, _I, _I, _P]),
    "vqa_reset_perm_index": (_L, [_U, _L, _I, _L, _L]),
    "vqa_mse_loss": (_I, [_P, _P, _P, _P, _P, _L, _P, _S, _P]),
    "vqa_mse_loss_workspace": (_S, [_L]),
    "vqa_adam_keras": (_I, [_P, _P, _P, _P, _L, _P, _F, _P, _F, _F, _F, _F, _P]),
    "vqa_lr_schedule": (_I, [_P, _P, _I, _F, _F, _F, _F, _P]),
    "vqa_counter_add": (_I, [_P, _L, _P]),
    "vqa_step_metrics": (_I, [_P, _P, _P, _I, _F, _P]),
    "vqa_synthetic_batch": (_I, [_P, _I, _L, _U, _I, _F, _P]),
    "vqa_embedding_fwd": (_I, [_P, _P, _P, _L, _I, _I, _I, _P]),
    "vqa_embedding_bwd": (_I, [_P, _P, _P, _L, _I, _I, _I, _P, _S, _P]),
    "vqa_embedding_bwd_workspace": (_S, [_L, _I, _I]),
    "vqa_layernorm_fwd": (_I, [_P, _P, _P, _P, _L, _I, _F, _I, _P]),
    "vqa_layernorm_bwd": (_I, [_P, _P, _P, _P, _P, _P, _L, _I, _F, _I, _P, _S, _P, _P]),
    "vqa_layernorm_bwd_workspace": (_S, [_L, _I]),
    "vqa_conv1d_bwd_weight_partials": (_I, [_P, _P, _P, _P] + _CONV + [_P, _S, _P, _P]),
    "vqa_conv1d_transpose_bwd_weight_partials": (_I, [_P, _P, _P, _P] + _CONVT + [_P, _S, _P, _P]),
    "vqa_reduce_partials": (_I, [_P, _I, _P]),
    "vqa_conv1d_bwd_data_weight": (_I, [_P, _P, _P, _P, _P, _P, _P] + _CONV + [_P, _S, _P, _P]),
    "vqa_conv1d_bwd_data_weight_workspace": (_S, _CONV),
    "vqa_spectral_loss": (_I, [_P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _I, _P, _S, _P]),
    "vqa_spectral_loss_workspace": (_S, [_I, _I, _P, _P, _P, _I, _I]),
    "vqa_stft_magnitude": (_I, [_P, _P, _I, _I, _I, _I, _I, _P]),
    "vqa_vq_argmin_split": (_I, [_P, _P, _P, _P, _P, _L, _I, _I, _P]),
    "vqa_vq_split_bf16x3": (_I, [_P, _P, _I, _I, _P]),
    "vqa_resblock_supported": (_I, [_I, _I, _I]),
    "vqa_resblock_fwd": (_I, [_P] * 7 + [_I] * 5 + [_P]),
    "vqa_resblock_bwd": (_I, [_P] * 11 + [_I] * 5 + [_P, _S, _P, _P]),
    "vqa_resblock_bwd_workspace": (_S, [_I] * 5),
    "vqa_dtail_supported": (_I, [_I] * 7),
    "vqa_dtail_workspace": (_S, [_I] * 5),
    "vqa_dtail_fwd": (_I, [_P] * 6 + [_I] * 5 + [_P, _S, _P]),
    "vqa_dtail_bwd": (_I, [_P] * 11 + [_I] * 5 + [_P, _S, _P]),
    "vqa_spectral_target_workspace": (_S, [_I, _I, _P, _P, _P, _I]),
    "vqa_spectral_target": (_I, [_P, _P, _S, _I, _I, _P, _P, _P, _I, _P]),
    "vqa_spectral_loss_target_workspace": (_S, [_I, _I, _P, _P, _P, _I, _I]),
    "vqa_spectral_loss_target": (_I, [_P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _I, _P, _S, _P]),
    # factorized-attention prior
    "vqa_seqlin_fwd": (_I, [_P, _L, _P, _P, _P, _L, _P, _L] + [_I] * 9 + [_P]),
    "vqa_seqlin_prep": (_I, [_P, _I, _I, _P]),
    "vqa_seqlin_fwd_prepped": (_I, [_P, _L, _P, _P, _P, _L, _P, _L] + [_I] * 8 + [_P]),
    "vqa_seqlin_fwd_ln_prepped": (_I, [_P, _L, _P, _P, ctypes.c_float, _P, _P, _P, _L, _P, _L] + [_I] * 7 + [_P]),
    "vqa_seqlin_wgrad_workspace": (_S, [_I] * 5),
    "vqa_seqlin_wgrad": (_I, [_P, _L, _P, _L, _P, _P] + [_I] * 6 + [_P, _S, _P, _P]),
    "vqa_prior_embed_fwd": (_I, [_P] * 6 + [_I] * 4 + [_F, _F, _U, _L, _P, _I, _P]),
    "vqa_colsum": (_I, [_P, _P, _I, _L, _L, _I, _I, _P]),
    "vqa_axpy": (_I, [_P, _P, _P, _L, _I, _P]),
    "vqa_dropout": (_I, [_P, _L, _F, _U, _U, _L, _P, _I, _P]),
    "vqa_scale_f32": (_I, [_P, _L, _F, _P]),
    "vqa_tf_mix": (_I, [_P, _P, _P, _P, _I, _I, _L, _F, _U, _U, _L, _P, _P]),
    "vqa_attn_fwd": (_I, [_P] * 6 + [_I] * 6 + [_F, _I, _P]),
    "vqa_attn_bwd": (_I, [_P] * 10 + [_I] * 6 + [_F, _I, _P]),
    "vqa_head_wt": (_I, [_P, _P, _I, _I, _I, _P]),
    "vqa_head_fwd": (_I, [_P] * 8 + [_L, _I, _I, _I, _P]),
    "vqa_head_bwd_workspace": (_S, [_L, _I, _I]),
    "vqa_head_bwd": (_I, [_P] * 5 + [_F, _P, _P, _P, _L, _I, _I, _I, _P, _S, _P, _P]),
    "vqa_rowsum_workspace": (_S, [_L, _L]),
    "vqa_rowsum": (_I, [_P, _L, _L, _F, _P, _P, _S, _P]),
    "vqa_prior_decode_cache_bytes": (_S, [_I, _I, _I]),
    "vqa_prior_decode": (_I, [_P, _I] + [_P] * 10 + [_S] + [_I] * 8 + [_L, _U, _P]),
}

_lib: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    """Load libvqa.so once. Raises ImportError if it has not been built (no fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libvqa.so not found at {LIB_PATH}; build it with `python -c "
                              f"'import __graft_entry__ as g; g.build()'` (there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        abi = L.vqa_abi_version() if hasattr(L, "vqa_abi_version") else 1
        if abi != ABI_VERSION:
            raise ImportError(f"{LIB_PATH} implements C-ABI revision {abi}, this binding needs {ABI_VERSION}: "
                              f"rebuild the library (argument lists differ between revisions)")
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    return lib().vqa_get_last_error().decode()


def _check(rc: int, what: str):
    if rc != 0:
        raise VQAError(f"{what} failed ({rc}): {last_error()}")


def ptr(t: Optional[torch.Tensor]):
    if t is None:
        return None
    if not t.is_cuda:
        raise VQAError("libvqa ops take device tensors only (got a CPU tensor)")
    if not t.is_contiguous():
        raise VQAError(f"libvqa ops take contiguous (N, T, C) tensors (got strides {t.stride()})")
    return ctypes.c_void_p(t.data_ptr())


# Test hook (tests/test_gpu_race.py, tools/cotenant.py inject): a callable run right before every libvqa launch is
# queued, on the launching thread with the launch's stream current — the race tests use it to put random spin
# delays in front of launches, so every cross-stream ordering the step relies on is exercised. None in the product.
launch_hook = None


def stream():
    if launch_hook is not None:
        launch_hook()
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.bfloat16:
        return BF16
    if dt == torch.float32:
        return F32
    raise VQAError(f"unsupported activation dtype {dt}")


def workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


# ---- host-only helpers (callable without a GPU) --------------------------------------------------
def same_pad_left(T_in: int, K: int, stride: int, dilation: int = 1) -> int:
    return lib().vqa_same_pad_left(T_in, K, stride, dilation)


def same_out_len(T_in: int, stride: int) -> int:
    return lib().vqa_same_out_len(T_in, stride)


def reset_perm_index(seed: int, counter: int, level: int, M: int, k: int) -> int:
    return lib().vqa_reset_perm_index(seed, counter, level, M, k)


# ---- device ops ------------------------------------------------------------------------------------
def conv1d_fwd(x, w, b, residual, y, B, T_in, T_out, C_in, C_out, K, stride, dilation, pad, flags, dtype):
    _check(lib().vqa_conv1d_fwd(ptr(x), ptr(w), ptr(b), ptr(residual), ptr(y), B, T_in, T_out, C_in, C_out, K,
                                stride, dilation, pad, flags, dtype, stream()), "vqa_conv1d_fwd")


def conv1d_bwd_data(dy, w, mask, residual, dx, B, T_in, T_out, C_in, C_out, K, stride, dilation, pad, flags, dtype):
    _check(lib().vqa_conv1d_bwd_data(ptr(dy), ptr(w), ptr(mask), ptr(residual), ptr(dx), B, T_in, T_out, C_in,
                                     C_out, K, stride, dilation, pad, flags, dtype, stream()), "vqa_conv1d_bwd_data")


def conv1d_bwd_weight(x, dy, dw, db, B, T_in, T_out, C_in, C_out, K, stride, dilation, pad, flags, dtype):
    n = lib().vqa_conv1d_bwd_weight_workspace(B, T_in, T_out, C_in, C_out, K, stride, dilation, pad, flags, dtype)
    ws = workspace(n, x.device)
    _check(lib().vqa_conv1d_bwd_weight(ptr(x), ptr(dy), ptr(dw), ptr(db), B, T_in, T_out, C_in, C_out, K, stride,
                                       dilation, pad, flags, dtype, ptr(ws), ws.numel(), stream()),
           "vqa_conv1d_bwd_weight")


class Deferred:
    """Collects deferred weight-gradient partials; flush() reduces them all in one launch."""

    def __init__(self):
        self.descs, self.keep = [], []

    def add(self, desc, ws):
        descs = desc if isinstance(desc, (list, tuple)) else [desc]
        self.descs.extend(descs)
        self.keep.append(ws)  # the partials must outlive the reduce launch

    def flush(self):
        if self.descs:
            arr = (PartialsDesc * len(self.descs))(*self.descs)
            _check(lib().vqa_reduce_partials(arr, len(self.descs), stream()), "vqa_reduce_partials")
        self.descs, self.keep = [], []


def conv1d_bwd_weight_deferred(x, dy, dw, db, B, T_in, T_out, C_in, C_out, K, stride, dilation, pad, flags, dtype,
                               deferred):
    n = lib().vqa_conv1d_bwd_weight_workspace(B, T_in, T_out, C_in, C_out, K, stride, dilation, pad, flags, dtype)
    ws = workspace(n, x.device)
    d = PartialsDesc()
    _check(lib().vqa_conv1d_bwd_weight_partials(ptr(x), ptr(dy), ptr(dw), ptr(db), B, T_in, T_out, C_in, C_out, K,
                                                stride, dilation, pad, flags, dtype, ptr(ws), ws.numel(),
                                                ctypes.byref(d), stream()), "vqa_conv1d_bwd_weight_partials")
    deferred.add(d, ws)


def conv1d_bwd_data_weight(dy, w, x, residual, dx, dw, db, B, T_in, T_out, C_in, C_out, K, stride, dilation, pad,
                           flags, dtype, deferred=None):
    """dx and (dw, db) of one Conv1D in one pass (vqa_conv1d_bwd_data_weight); `x` is the conv input (its
    ReLU' mask with VQA_PRE_RELU). With `deferred` the weight-gradient reduction joins its batch."""
    n = lib().vqa_conv1d_bwd_data_weight_workspace(B, T_in, T_out, C_in, C_out, K, stride, dilation, pad, flags,
                                                    dtype)
    ws = workspace(n, x.device)
    d = PartialsDesc() if deferred is not None else None
    _check(lib().vqa_conv1d_bwd_data_weight(ptr(dy), ptr(w), ptr(x), ptr(residual), ptr(dx), ptr(dw), ptr(db), B,
                                            T_in, T_out, C_in, C_out, K, stride, dilation, pad, flags, dtype,
                                            ptr(ws), ws.numel(), ctypes.byref(d) if d is not None else None,
                                            stream()), "vqa_conv1d_bwd_data_weight")
    if deferred is not None:
        deferred.add(d, ws)


def dtail_supported(C, Cu, K_up, stride_up, K_out, C_out, dtype) -> bool:
    return bool(lib().vqa_dtail_supported(C, Cu, K_up, stride_up, K_out, C_out, dtype))


def dtail_fwd(h, w_up, b_up, w_out, b_out, y):
    """encdec.py:67-68 (last Conv1DTranspose) + :148 (output Conv1D) composed: h (B, T, 32) -> y (B, 2T, 1)
    fp32 (vqa_dtail_fwd)."""
    B, T, C = h.shape
    dt = dtype_code(h.dtype)
    Cu = w_up.shape[1]
    ws = workspace(lib().vqa_dtail_workspace(B, T, C, Cu, dt), h.device)
    _check(lib().vqa_dtail_fwd(ptr(h), ptr(w_up), ptr(b_up), ptr(w_out), ptr(b_out), ptr(y), B, T, C, Cu, dt, ptr(ws),
                               ws.numel(), stream()), "vqa_dtail_fwd")


def dtail_bwd(dy, h, w_up, b_up, w_out, b_out, dh, dw_up, db_up, dw_out, db_out):
    """Backward of dtail_fwd: dh and the gradients of both layers' kernels and biases (written)."""
    B, T, C = h.shape
    dt = dtype_code(h.dtype)
    Cu = w_up.shape[1]
    ws = workspace(lib().vqa_dtail_workspace(B, T, C, Cu, dt), h.device)
    _check(lib().vqa_dtail_bwd(ptr(dy), ptr(h), ptr(w_up), ptr(b_up), ptr(w_out), ptr(b_out), ptr(dh), ptr(dw_up),
                               ptr(db_up), ptr(dw_out), ptr(db_out), B, T, C, Cu, dt, ptr(ws), ws.numel(), stream()),
           "vqa_dtail_bwd")


def resblock_supported(C, dilation, dtype) -> bool:
    return bool(lib().vqa_resblock_supported(C, dilation, dtype))


def resblock_fwd(x, wa, ba, wb, bb, y, dilation, h_out=None):
    """resnet.py:7-29 forward, fused (vqa_resblock_fwd); x, y, h_out (B, T, 32) in the compute dtype."""
    B, T, C = x.shape
    _check(lib().vqa_resblock_fwd(ptr(x), ptr(wa), ptr(ba), ptr(wb), ptr(bb), ptr(y), ptr(h_out), B, T, C, dilation,
                                  dtype_code(x.dtype), stream()), "vqa_resblock_fwd")


def resblock_bwd(dy, x, wa, ba, wb, bb, dx, dwa, dba, dwb, dbb, dilation, deferred=None):
    """Backward of the fused block (h recomputed from x): dx and the four weight gradients."""
    B, T, C = x.shape
    dt = dtype_code(x.dtype)
    ws = workspace(lib().vqa_resblock_bwd_workspace(B, T, C, dilation, dt), x.device)
    descs = (PartialsDesc * 2)() if deferred is not None else None
    _check(lib().vqa_resblock_bwd(ptr(dy), ptr(x), ptr(wa), ptr(ba), ptr(wb), ptr(bb), ptr(dx), ptr(dwa), ptr(dba),
                                  ptr(dwb), ptr(dbb), B, T, C, dilation, dt, ptr(ws), ws.numel(), descs, stream()),
           "vqa_resblock_bwd")
    if deferred is not None:
        deferred.add([descs[0], descs[1]], ws)


def conv1d_transpose_bwd_weight_deferred(x, dy, dw, db, B, T_in, T_out, C_in, C_out, K, stride, pad, flags, dtype,
                                         deferred):
    n = lib().vqa_conv1d_transpose_bwd_weight_workspace(B, T_in, T_out, C_in, C_out, K, stride, pad, flags, dtype)
    ws = workspace(n, x.device)
    d = PartialsDesc()
    _check(lib().vqa_conv1d_transpose_bwd_weight_partials(ptr(x), ptr(dy), ptr(dw), ptr(db), B, T_in, T_out, C_in,
                                                          C_out, K, stride, pad, flags, dtype, ptr(ws), ws.numel(),
                                                          ctypes.byref(d), stream()),
           "vqa_conv1d_transpose_bwd_weight_partials")
    deferred.add(d, ws)


def conv1d_transpose_fwd(x, w, b, residual, y, B, T_in, T_out, C_in, C_out, K, stride, pad, flags, dtype):
    _check(lib().vqa_conv1d_transpose_fwd(ptr(x), ptr(w), ptr(b), ptr(residual), ptr(y), B, T_in, T_out, C_in,
                                          C_out, K, stride, pad, flags, dtype, stream()), "vqa_conv1d_transpose_fwd")


def conv1d_transpose_bwd_data(dy, w, mask, residual, dx, B, T_in, T_out, C_in, C_out, K, stride, pad, flags, dtype):
    _check(lib().vqa_conv1d_transpose_bwd_data(ptr(dy), ptr(w), ptr(mask), ptr(residual), ptr(dx), B, T_in, T_out,
                                               C_in, C_out, K, stride, pad, flags, dtype, stream()),
           "vqa_conv1d_transpose_bwd_data")


def conv1d_transpose_bwd_weight(x, dy, dw, db, B, T_in, T_out, C_in, C_out, K, stride, pad, flags, dtype):
    n = lib().vqa_conv1d_transpose_bwd_weight_workspace(B, T_in, T_out, C_in, C_out, K, stride, pad, flags, dtype)
    ws = workspace(n, x.device)
    _check(lib().vqa_conv1d_transpose_bwd_weight(ptr(x), ptr(dy), ptr(dw), ptr(db), B, T_in, T_out, C_in, C_out, K,
                                                 stride, pad, flags, dtype, ptr(ws), ws.numel(), stream()),
           "vqa_conv1d_transpose_bwd_weight")


def vq_sqnorm(E, esq):
    D, K = E.shape
    _check(lib().vqa_vq_sqnorm(ptr(E), ptr(esq), D, K, stream()), "vqa_vq_sqnorm")


def vq_argmin(z, E, esq, idx, min_dist=None):
    N, D = z.shape
    K = E.shape[1]
    _check(lib().vqa_vq_argmin(ptr(z), ptr(E), ptr(esq), ptr(idx), ptr(min_dist), N, D, K, dtype_code(z.dtype),
                               stream()), "vqa_vq_argmin")


def vq_split_bf16x3(E, E3):
    D, K = E.shape
    if tuple(E3.shape) != (K, 3, D) or E3.dtype != torch.bfloat16:
        raise VQAError(f"vq_split_bf16x3: E3 must be ({K}, 3, {D}) bf16")
    _check(lib().vqa_vq_split_bf16x3(ptr(E), ptr(E3), D, K, stream()), "vqa_vq_split_bf16x3")


def vq_argmin_split(z, E3, esq, idx, min_dist=None):
    N, D = z.shape
    K = E3.shape[0]
    if z.dtype != torch.bfloat16:
        raise VQAError("vq_argmin_split takes bf16 z")
    _check(lib().vqa_vq_argmin_split(ptr(z), ptr(E3), ptr(esq), ptr(idx), ptr(min_dist), N, D, K, stream()),
           "vqa_vq_argmin_split")


def vq_quantize(z, ET, idx, q_st, commit_out, m_sumT, n_sum, beta):
    N, D = z.shape
    K = ET.shape[0]
    dt = dtype_code(z.dtype)
    ws = workspace(lib().vqa_vq_quantize_workspace(N, D, K, dt), z.device)
    _check(lib().vqa_vq_quantize(ptr(z), ptr(ET), ptr(idx), ptr(q_st), ptr(commit_out), ptr(m_sumT), ptr(n_sum), N,
                                 D, K, beta, dt, ptr(ws), ws.numel(), stream()), "vqa_vq_quantize")


def vq_backward(dq, z, ET, idx, dz, scale):
    N, D = z.shape
    _check(lib().vqa_vq_backward(ptr(dq), ptr(z), ptr(ET), ptr(idx), ptr(dz), scale, N, D, dtype_code(z.dtype),
                                 stream()), "vqa_vq_backward")


def vq_reset_rows(z, RT, row_offset, N_global, seed, counter, level):
    N, D = z.shape
    K = RT.shape[0]
    _check(lib().vqa_vq_reset_rows(ptr(z), ptr(RT), N, row_offset, N_global, D, K, seed, ptr(counter), level,
                                   dtype_code(z.dtype), stream()), "vqa_vq_reset_rows")


def vq_ema_apply(E, ET, m_t, N_t, m_sumT, n_sum, RT, gamma, omg, thresh, metrics, counter, esq=None, E3=None):
    """EMA + dead-code reset; with esq / E3 also |e|^2 and the bf16 planes of the new codebook (same pass)."""
    D, K = E.shape
    if E3 is not None and (E3.dtype != torch.bfloat16 or tuple(E3.shape) != (K, 3, D)):
        raise VQAError(f"vq_ema_apply: E3 must be ({K}, 3, {D}) bf16")
    _check(lib().vqa_vq_ema_apply_derived(ptr(E), ptr(ET), ptr(m_t), ptr(N_t), ptr(m_sumT), ptr(n_sum), ptr(RT), gamma,
                                          omg, thresh, ptr(metrics), ptr(counter), ptr(esq), ptr(E3), D, K, stream()),
           "vqa_vq_ema_apply_derived")


def mse_loss(x, r, extra, dr, loss_out):
    n = x.numel()
    ws = workspace(lib().vqa_mse_loss_workspace(n), x.device)
    _check(lib().vqa_mse_loss(ptr(x), ptr(r), ptr(extra), ptr(dr), ptr(loss_out), n, ptr(ws), ws.numel(), stream()),
           "vqa_mse_loss")


def adam_keras(w, g, m, v, step, lr, beta1, beta2, eps, grad_scale, lr_dev=None):
    _check(lib().vqa_adam_keras(ptr(w), ptr(g), ptr(m), ptr(v), w.numel(), ptr(step), float(lr), ptr(lr_dev), beta1,
                                beta2, eps, grad_scale, stream()), "vqa_adam_keras")


def lr_schedule(step, lr_out, kind, p):
    p = list(p) + [0.0] * (4 - len(p))
    _check(lib().vqa_lr_schedule(ptr(step), ptr(lr_out), int(kind), *[float(v) for v in p[:4]], stream()),
           "vqa_lr_schedule")


def step_metrics(loss_slots, vq_metrics, macc, levels, scale):
    _check(lib().vqa_step_metrics(ptr(loss_slots), ptr(vq_metrics), ptr(macc), levels, scale, stream()),
           "vqa_step_metrics")


def synthetic_batch(x, seed, rank=0, sample_rate=44100.0):
    """x: (B, T) or (B, T, 1) fp32 device tensor, filled in place (vqa_synthetic_batch)."""
    B, T = x.shape[0], x.numel() // x.shape[0]
    if x.dtype != torch.float32:
        raise VQAError("synthetic_batch fills an fp32 tensor")
    _check(lib().vqa_synthetic_batch(ptr(x), B, T, seed, rank, sample_rate, stream()), "vqa_synthetic_batch")


def embedding_fwd(table, idx, out):
    """src/conditioner/conditioners.py:64 layers.Embedding: out (..., D) = table[idx] (vqa_embedding_fwd)."""
    K, D = table.shape
    N = idx.numel()
    if idx.dtype != torch.int64 or out.shape[-1] != D or out.numel() != N * D:
        raise VQAError("embedding_fwd: idx int64 (...), out (..., D)")
    _check(lib().vqa_embedding_fwd(ptr(table), ptr(idx), ptr(out), N, D, K, dtype_code(out.dtype), stream()),
           "vqa_embedding_fwd")


def embedding_bwd(dy, idx, dtable):
    """dtable[k] += sum of dy rows with idx == k, fixed order (vqa_embedding_bwd)."""
    K, D = dtable.shape
    N = idx.numel()
    ws = workspace(lib().vqa_embedding_bwd_workspace(N, D, K), dy.device)
    _check(lib().vqa_embedding_bwd(ptr(dy), ptr(idx), ptr(dtable), N, D, K, dtype_code(dy.dtype), ptr(ws), ws.numel(),
                                   stream()), "vqa_embedding_bwd")


def layernorm_fwd(x, gamma, beta, y, eps):
    C = x.shape[-1]
    _check(lib().vqa_layernorm_fwd(ptr(x), ptr(gamma), ptr(beta), ptr(y), x.numel() // C, C, eps, dtype_code(x.dtype),
                                   stream()), "vqa_layernorm_fwd")


def layernorm_bwd(x, dy, gamma, dx, dgamma, dbeta, eps, deferred=None):
    C = x.shape[-1]
    rows = x.numel() // C
    ws = workspace(lib().vqa_layernorm_bwd_workspace(rows, C), x.device)
    d = PartialsDesc() if deferred is not None else None
    _check(lib().vqa_layernorm_bwd(ptr(x), ptr(dy), ptr(gamma), ptr(dx), ptr(dgamma), ptr(dbeta), rows, C, eps,
                                   dtype_code(x.dtype), ptr(ws), ws.numel(), ctypes.byref(d) if d is not None else None,
                                   stream()), "vqa_layernorm_bwd")
    if deferred is not None:
        deferred.add(d, ws)


def counter_add(counter, delta=1):
    _check(lib().vqa_counter_add(ptr(counter), delta, stream()), "vqa_counter_add")


def _int_array(vals):
    return (ctypes.c_int * len(vals))(*[int(v) for v in vals])


def spectral_loss_workspace(B, T, n_fft, hop, win, with_grad=True) -> int:
    n = lib().vqa_spectral_loss_workspace(B, T, _int_array(n_fft), _int_array(hop), _int_array(win), len(n_fft),
                                          1 if with_grad else 0)
    if n == 0:
        raise VQAError(f"spectral_loss: bad shape B={B} T={T} n_fft={n_fft} hop={hop} win={win}")
    return n


def spectral_loss(x, r, loss_out, dr, item_loss, n_fft, hop, win, ws=None):
    """x, r, dr: (B, T) fp32 device tensors; loss_out: 1-element fp32. dr / item_loss may be None."""
    B, T = x.shape[0], x.numel() // x.shape[0]
    nres = len(n_fft)
    if ws is None:
        ws = workspace(spectral_loss_workspace(B, T, n_fft, hop, win, dr is not None), x.device)
    _check(lib().vqa_spectral_loss(ptr(x), ptr(r), ptr(loss_out), ptr(dr), ptr(item_loss), B, T, _int_array(n_fft),
                                   _int_array(hop), _int_array(win), nres, ptr(ws), ws.numel(), stream()),
           "vqa_spectral_loss")


def spectral_target(x, n_fft, hop, win):
    """Tables + |S_x| of every resolution for a (B, T) fp32 target -> a uint8 device buffer."""
    B, T = x.shape[0], x.numel() // x.shape[0]
    a = (_int_array(n_fft), _int_array(hop), _int_array(win))
    n = lib().vqa_spectral_target_workspace(B, T, *a, len(n_fft))
    if n == 0:
        raise VQAError(f"spectral_target: bad shape B={B} T={T} n_fft={n_fft} hop={hop} win={win}")
    tg = workspace(n, x.device)
    _check(lib().vqa_spectral_target(ptr(x), ptr(tg), tg.numel(), B, T, *a, len(n_fft), stream()),
           "vqa_spectral_target")
    return tg


def spectral_loss_target_workspace(B, T, n_fft, hop, win, with_grad=True) -> int:
    n = lib().vqa_spectral_loss_target_workspace(B, T, _int_array(n_fft), _int_array(hop), _int_array(win),
                                                 len(n_fft), 1 if with_grad else 0)
    if n == 0:
        raise VQAError(f"spectral_loss_target: bad shape B={B} T={T} n_fft={n_fft} hop={hop} win={win}")
    return n


def spectral_loss_target(target, r, loss_out, dr, item_loss, n_fft, hop, win, ws=None):
    """The spectral loss of r (B, T) against a spectral_target buffer; dr / item_loss may be None."""
    B, T = r.shape[0], r.numel() // r.shape[0]
    a = (_int_array(n_fft), _int_array(hop), _int_array(win))
    if ws is None:
        ws = workspace(spectral_loss_target_workspace(B, T, n_fft, hop, win, dr is not None), r.device)
    _check(lib().vqa_spectral_loss_target(ptr(target), ptr(r), ptr(loss_out), ptr(dr), ptr(item_loss), B, T, *a,
                                          len(n_fft), ptr(ws), ws.numel(), stream()), "vqa_spectral_loss_target")


def stft_magnitude(x, mag, n_fft, hop, win):
    B, T = x.shape[0], x.numel() // x.shape[0]
    _check(lib().vqa_stft_magnitude(ptr(x), ptr(mag), B, T, n_fft, hop, win, stream()), "vqa_stft_magnitude")


# ---- factorized-attention prior (vqa_prior.hip) -----------------------------------------------------
def rptr(t: torch.Tensor):
    """(pointer, row stride) of a row-strided view (last dim contiguous, uniform row stride): column slices
    such as qkv[..., 0:32] of a (N, T, 96) tensor."""
    if not t.is_cuda:
        raise VQAError("libvqa ops take device tensors only (got a CPU tensor)")
    if t.stride(-1) != 1:
        raise VQAError("row-strided view needs a contiguous last dimension")
    ld = t.stride(-2) if t.dim() >= 2 else t.shape[-1]
    for d in range(t.dim() - 2):
        if t.stride(d) != t.stride(d + 1) * t.shape[d + 1]:
            raise VQAError(f"view with strides {t.stride()} is not row-strided")
    return ctypes.c_void_p(t.data_ptr()), ld


def seqlin_fwd(x, w, b, y, T, taps=1, dir=-1, wtrans=False, residual=None, accumulate=False):
    """vqa_seqlin_fwd on (nseq*T, K) rows -> (nseq*T, N) rows. w: (taps, K, N) (wtrans: (taps, N, K)) or (K, N)."""
    px, ldx = rptr(x)
    py, ldy = rptr(y)
    pr, ldr = rptr(residual) if residual is not None else (None, 0)
    K, N = x.shape[-1], y.shape[-1]
    rows = x.numel() // K
    _check(lib().vqa_seqlin_fwd(px, ldx, ptr(w), ptr(b), pr, ldr, py, ldy, rows // T, T, K, N, taps, dir,
                                int(bool(wtrans)), int(bool(accumulate)), dtype_code(x.dtype), stream()),
           "vqa_seqlin_fwd")


class SeqlinPrepDesc(ctypes.Structure):
    """vqa_seqlin_prep_desc (include/vqa.h)."""
    _fields_ = [("w", ctypes.c_void_p), ("out", ctypes.c_void_p), ("taps", ctypes.c_int), ("K", ctypes.c_int),
                ("N", ctypes.c_int), ("wtrans", ctypes.c_int)]


def seqlin_prep(descs, dtype):
    """One launch converting a list of (w fp32 tensor, out tensor, taps, K, N, wtrans) to [taps][N][K] images."""
    arr = (SeqlinPrepDesc * len(descs))(*[SeqlinPrepDesc(ptr(w).value, ptr(o).value, t, k, n, int(bool(tr)))
                                         for (w, o, t, k, n, tr) in descs])
    _check(lib().vqa_seqlin_prep(arr, len(descs), dtype_code(dtype), stream()), "vqa_seqlin_prep")


def seqlin_fwd_prepped(x, wp, b, y, T, taps=1, dir=-1, residual=None, accumulate=False):
    """vqa_seqlin_fwd_prepped: wp = (taps, N, K) image in the activation dtype (seqlin_prep)."""
    px, ldx = rptr(x)
    py, ldy = rptr(y)
    pr, ldr = rptr(residual) if residual is not None else (None, 0)
    K, N = x.shape[-1], y.shape[-1]
    rows = x.numel() // K
    _check(lib().vqa_seqlin_fwd_prepped(px, ldx, ptr(wp), ptr(b), pr, ldr, py, ldy, rows // T, T, K, N, taps, dir,
                                        int(bool(accumulate)), dtype_code(x.dtype), stream()),
           "vqa_seqlin_fwd_prepped")


def seqlin_fused_ln_ok(x, K):
    """vqa_seqlin_fwd_ln_prepped's domain: bf16 activations with K = 128 channels."""
    return x.dtype == torch.bfloat16 and K == 128


def seqlin_fwd_ln_prepped(x, gamma, beta, eps, wp, b, y, T, taps=1, dir=-1, residual=None):
    """vqa_seqlin_fwd_ln_prepped: seqlin_fwd_prepped(LayerNorm(x)) in one launch (bf16, K = 128)."""
    px, ldx = rptr(x)
    py, ldy = rptr(y)
    pr, ldr = rptr(residual) if residual is not None else (None, 0)
    K, N = x.shape[-1], y.shape[-1]
    rows = x.numel() // K
    _check(lib().vqa_seqlin_fwd_ln_prepped(px, ldx, ptr(gamma), ptr(beta), float(eps), ptr(wp), ptr(b), pr, ldr, py,
                                           ldy, rows // T, T, K, N, taps, dir, dtype_code(x.dtype), stream()),
           "vqa_seqlin_fwd_ln_prepped")


def seqlin_wgrad(x, dy, dw, db, T, taps=1, deferred=None):
    px, ldx = rptr(x)
    pd, ldd = rptr(dy)
    K, N = x.shape[-1], dy.shape[-1]
    nseq = (x.numel() // K) // T
    ws = workspace(lib().vqa_seqlin_wgrad_workspace(nseq, T, K, N, taps), x.device)
    d = PartialsDesc() if deferred is not None else None
    _check(lib().vqa_seqlin_wgrad(px, ldx, pd, ldd, ptr(dw), ptr(db), nseq, T, K, N, taps, dtype_code(x.dtype),
                                  ptr(ws), ws.numel(), ctypes.byref(d) if d is not None else None, stream()),
           "vqa_seqlin_wgrad")
    if deferred is not None:
        deferred.add(d, ws)


def prior_embed_fwd(table, pos, tokens, out, scale, ycond=None, xcond=None, rate=0.0, seed=0, counter=None,
                    elem_offset=0):
    N, T = tokens.shape
    bins, W = table.shape
    _check(lib().vqa_prior_embed_fwd(ptr(table), ptr(pos), ptr(tokens), ptr(ycond), ptr(xcond), ptr(out), N, T, W,
                                     bins, scale, rate, seed, int(elem_offset), ptr(counter), dtype_code(out.dtype),
                                     stream()),
           "vqa_prior_embed_fwd")


def colsum(x, out, nout, ostride, inner, accumulate=False):
    _check(lib().vqa_colsum(ptr(x), ptr(out), nout, ostride, inner, int(bool(accumulate)), dtype_code(x.dtype),
                            stream()), "vqa_colsum")


def axpy(x, y, z):
    _check(lib().vqa_axpy(ptr(x), ptr(y), ptr(z), x.numel(), dtype_code(x.dtype), stream()), "vqa_axpy")


EMB_DROPOUT_SALT = 0x454D42  # VQA_EMB_DROPOUT_SALT: vqa_prior_embed_fwd's dropout mask is vqa_dropout's with this salt


def dropout_(x, rate, seed, salt, counter=None, elem_offset=0):
    """keras Dropout in place; elem_offset = the global flat index of x[0] (data parallel: rank * x.numel())."""
    _check(lib().vqa_dropout(ptr(x), x.numel(), rate, seed, salt, int(elem_offset), ptr(counter), dtype_code(x.dtype),
                             stream()),
           "vqa_dropout")


def scale_f32_(x, s):
    _check(lib().vqa_scale_f32(ptr(x), x.numel(), s, stream()), "vqa_scale_f32")


def tf_mix(codes, amax, mask, out, start, rate=0.0, seed=0, step=0, counter=None, row_offset=0):
    N, T = codes.shape
    _check(lib().vqa_tf_mix(ptr(codes), ptr(amax), ptr(mask), ptr(out), N, T, start, rate, seed, step, row_offset,
                            ptr(counter), stream()), "vqa_tf_mix")


def attn_fwd(q, k, v, o, lse, mode, l, heads, scale, vbias=None):
    N, T, C = q.shape
    _check(lib().vqa_attn_fwd(ptr(q), ptr(k), ptr(v), ptr(o), ptr(lse), ptr(vbias), N, T, heads, C // heads, l, mode,
                              scale, dtype_code(q.dtype), stream()), "vqa_attn_fwd")


def attn_bwd(q, k, v, o, lse, dout, dsum, dq, dk, dv, mode, l, heads, scale):
    N, T, C = q.shape
    _check(lib().vqa_attn_bwd(ptr(q), ptr(k), ptr(v), ptr(o), ptr(lse), ptr(dout), ptr(dsum), ptr(dq), ptr(dk),
                              ptr(dv), N, T, heads, C // heads, l, mode, scale, dtype_code(q.dtype), stream()),
           "vqa_attn_bwd")


def head_wt(w, wt):
    K, V = w.shape
    _check(lib().vqa_head_wt(ptr(w), ptr(wt), K, V, dtype_code(wt.dtype), stream()), "vqa_head_wt")


def head_fwd(x, wt, bias, lse, amax=None, targets=None, loss_row=None, correct=None):
    K = x.shape[-1]
    M = x.numel() // K
    _check(lib().vqa_head_fwd(ptr(x), ptr(wt), ptr(bias), ptr(targets), ptr(lse), ptr(amax), ptr(loss_row),
                              ptr(correct), M, K, wt.shape[0], dtype_code(x.dtype), stream()), "vqa_head_fwd")


def head_bwd(x, wt, bias, targets, lse, inv_count, dx, dw, db, deferred=None):
    K = x.shape[-1]
    M = x.numel() // K
    V = wt.shape[0]
    ws = workspace(lib().vqa_head_bwd_workspace(M, K, V), x.device)
    d = PartialsDesc() if deferred is not None else None
    _check(lib().vqa_head_bwd(ptr(x), ptr(wt), ptr(bias), ptr(targets), ptr(lse), inv_count, ptr(dx), ptr(dw),
                              ptr(db), M, K, V, dtype_code(x.dtype), ptr(ws), ws.numel(),
                              ctypes.byref(d) if d is not None else None, stream()), "vqa_head_bwd")
    if deferred is not None:
        deferred.add(d, ws)


def rowsum(x, rows, n, scale, out):
    ws = workspace(lib().vqa_rowsum_workspace(rows, n), x.device)
    _check(lib().vqa_rowsum(ptr(x), rows, n, scale, ptr(out), ptr(ws), ws.numel(), stream()), "vqa_rowsum")


class PriorLayerDesc(ctypes.Structure):
    """vqa_prior_layer (include/vqa.h)."""
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "ln1_gamma", "ln1_beta", "qkv_kernel", "qkv_bias", "query_kernel", "query_bias", "key_kernel", "key_bias",
        "value_kernel", "value_bias", "out_kernel", "out_bias", "proj_kernel", "proj_bias", "ln2_gamma", "ln2_beta",
        "mlp_kernel", "mlp_bias")] + [("attn_type", ctypes.c_int)]


def prior_decode(layers, emb, pos, out_w, out_b, tokens, cache, steps, ctx, heads, blocks, start, seed, ycond=None,
                 xcond=None, forced=None, logits=None, bins=None):
    """out_w (width, ld) / out_b (ld,) with ld a multiple of 4 >= bins (zero-padded columns are never sampled)."""
    N = tokens.shape[0]
    bins = out_w.shape[1] if bins is None else int(bins)
    arr = (PriorLayerDesc * len(layers))(*layers)
    _check(lib().vqa_prior_decode(arr, len(layers), ptr(emb), ptr(pos), ptr(out_w), ptr(out_b), ptr(ycond),
                                  ptr(xcond), ptr(forced), ptr(logits), ptr(tokens), ptr(cache), cache.numel(), N,
                                  steps, ctx, emb.shape[1], heads, blocks, bins, out_w.shape[1], start, seed, stream()),
           "vqa_prior_decode")
