"""Data-parallel exchange for the VQ-VAE train step (one process per GPU, RCCL over xGMI).

The reference trains on one device (vqvae.py:111-146). Split by batch items over W ranks, the step is
exactly the single-device step at global batch W*B provided:
  - gradients of the per-rank MEAN losses are averaged (recon / commitment / spectral are all means
    over items or elements of equal-size shards)         -> all_reduce(SUM) then scale 1/W;
  - the codebook EMA statistics m_sum (VectorQuantizer.py:123) and n_sum (:124) are SUMS over rows
                                                          -> all_reduce(SUM), applied as is;
  - the dead-code reset candidates (shuffle(tile(flat))[:K], :137) are rows of the GLOBAL flattened
    batch (global row = rank * N_local + local row): each rank writes the candidate rows it owns and
    zeros elsewhere                                       -> all_reduce(SUM) assembles R exactly.
All of it is ONE flat fp32 bucket [grads | per-level (m_sumT, n_sum, RT) | per-level losses], so a step
has exactly one collective; with ~5.5 MB at cfg2 it is latency-bound on xGMI (~tens of microseconds).
"""
from __future__ import annotations

from typing import Dict, Sequence

import os

import torch
import torch.distributed as dist

# diagnosis only (tools/dp_diag.py, round-3 failure study): hand gloo the device bucket as the RCCL path does
_GLOO_DEVICE = os.environ.get("VQA_DP_GLOO_DEVICE") == "1"


def bucket_layout(n_params: int, stats_sizes: Sequence[int], levels: int, align: int = 64) -> Dict[str, object]:
    """Offsets of the regions of the all-reduce bucket (grads padded to `align` floats)."""
    P = (n_params + align - 1) // align * align
    stats = []
    off = P
    for n in stats_sizes:
        stats.append((off, off + n))
        off += n
    losses = (off, off + 3 * levels)
    return {"grads": (0, P), "n_params": n_params, "stats": stats, "losses": losses, "total": losses[1]}


def vq_stats_slices(K: int, D: int):
    """Inside one level's stats region: m_sumT (K*D), n_sum (K), RT (K*D)."""
    return {"m_sumT": (0, K * D), "n_sum": (K * D, K * D + K), "RT": (K * D + K, 2 * K * D + K)}


def world_size(group=None) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def rank(group=None) -> int:
    return dist.get_rank(group) if dist.is_available() and dist.is_initialized() else 0


def exchange(bucket: torch.Tensor, group=None) -> int:
    """Sum the bucket over ranks (no-op on one rank). Returns the world size (grad scale = 1/W)."""
    w = world_size(group)
    if w > 1:
        # RCCL over xGMI ("nccl"): ordered on the current stream, on the device bucket. The gloo rehearsal
        # backend (tests, bench under VQA_DIST_BACKEND=gloo) stages the bucket through host memory itself: a
        # blocking copy out on the producer stream (which has joined the levels' streams), the CPU all_reduce,
        # and a copy back on the same stream. Handing gloo the device bucket (its own pinned staging on a pool
        # stream behind an event) left the 2-rank bf16 graph-warm-up test with a sum that missed part of the
        # last-produced gradients (level 2, encoder block 0) in a few runs, even after a host sync first.
        if bucket.is_cuda and dist.get_backend(group) == dist.Backend.GLOO and not _GLOO_DEVICE:
            host = bucket.to("cpu")  # synchronous: waits for the producer stream
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
            bucket.copy_(host)
            return w
        dist.all_reduce(bucket, op=dist.ReduceOp.SUM, group=group)
    return w


def global_row_range(n_local: int, group=None):
    """(row_offset, N_global) of this rank's VQ rows in the global flattened batch."""
    return rank(group) * n_local, world_size(group) * n_local
