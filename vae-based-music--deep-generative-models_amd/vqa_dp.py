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

import torch
import torch.distributed as dist

# Test hook (tests/test_gpu_rccl.py): take the data-parallel path — the exchange's collective on the device bucket,
# the EMA after it, two graphs around it — even in a process group of ONE rank, so the RCCL branch runs on a
# one-GPU box. Off in the product: at world size 1 the step needs no exchange.
FORCE_COLLECTIVE = False


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


def active(group=None) -> bool:
    """Does the step take the data-parallel path (exchange, EMA after it, split graphs)?"""
    return world_size(group) > 1 or (FORCE_COLLECTIVE and dist.is_available() and dist.is_initialized())


def exchange(bucket: torch.Tensor, group=None) -> int:
    """Sum the bucket over ranks (no-op on one rank). Returns the world size (grad scale = 1/W).

    RCCL over xGMI ("nccl"): one all_reduce on the device bucket, queued on the current (producer) stream — which
    has joined the levels' streams — so it reads the finished gradients and every later launch on that stream
    reads the sum. The gloo rehearsal backend (the tests, bench under VQA_DIST_BACKEND=gloo) gets the bucket staged
    through host memory here: a blocking copy out on the producer stream, the CPU all_reduce, a copy back on the
    same stream (gloo's own device staging runs on a side stream of its own; host staging keeps this one order)."""
    w = world_size(group)
    if active(group):
        if bucket.is_cuda and dist.get_backend(group) == dist.Backend.GLOO:
            host = bucket.to("cpu")  # synchronous: waits for the producer stream
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
            bucket.copy_(host)
            return w
        dist.all_reduce(bucket, op=dist.ReduceOp.SUM, group=group)
    return w


def global_row_range(n_local: int, group=None):
    """(row_offset, N_global) of this rank's VQ rows in the global flattened batch."""
    return rank(group) * n_local, world_size(group) * n_local
