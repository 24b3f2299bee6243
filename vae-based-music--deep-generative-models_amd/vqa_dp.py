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
is summed by one collective by default; with ~7 MB at cfg2 it is latency-bound on xGMI (tens of µs).

Overlapped form (VQVAE(overlap_exchange=True) / VQA_DP_OVERLAP=1; off by default): the levels' chains are independent, so each
level's share of the bucket — its layers' gradient range and its VQ statistics (`level_regions`) — is summed as
soon as that level's backward ends, on the level's own stream, while the other levels still compute (SURVEY.md
§8e: "the all-reduce overlaps with the backward pass of earlier levels"); the level's codebook EMA follows on
that stream and only the 3*levels loss floats are summed after the join. Same sums (elementwise), 2*levels + 1
collectives instead of one. On RCCL these are issued straight to the process group's communicator
(`ncclAllReduce` from the librccl torch itself loaded) on the level's own stream, so they can be captured into
the step's hipGraph: a collective captured through torch.distributed leaves its completion events with the
process group's watchdog, which queries them while the capture is open and aborts (hipErrorCapturedEvent,
PyTorch 2.10 / ROCm 7), and a collective on a side stream forked from a level stream crashes capture_end
(tools/capture_fork_probe.py: every nested-fork form segfaults, the level-stream form replays right). RCCL runs
one communicator's operations in the order they were issued, whatever streams they are queued on (its internal
strong stream, in eager mode and in captured graphs alike), and every rank issues the same sequence.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Dict, List, Sequence, Tuple

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


def device_side(group=None) -> bool:
    """Is the process group's backend a device-side one (RCCL, "nccl")?"""
    return dist.get_backend(group) == dist.Backend.NCCL


def host_staged(bucket: torch.Tensor, group=None) -> bool:
    """Does `exchange` stage this bucket through host memory (gloo with a device bucket)? Such an exchange
    blocks the host and cannot be captured into a graph."""
    return bool(bucket.is_cuda and dist.get_backend(group) == dist.Backend.GLOO)


def exchange(bucket: torch.Tensor, group=None) -> int:
    """Sum the bucket over ranks (no-op on one rank). Returns the world size (grad scale = 1/W).

    RCCL over xGMI ("nccl"): one all_reduce on the device bucket, queued on the current (producer) stream — which
    has joined the levels' streams — so it reads the finished gradients and every later launch on that stream
    reads the sum. The gloo rehearsal backend (the tests, bench under VQA_DIST_BACKEND=gloo) gets the bucket staged
    through host memory here: a blocking copy out on the producer stream, the CPU all_reduce, a copy back on the
    same stream (gloo's own device staging runs on a side stream of its own; host staging keeps this one order)."""
    w = world_size(group)
    if active(group):
        if host_staged(bucket, group):
            host = bucket.to("cpu")  # synchronous: waits for the producer stream
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
            bucket.copy_(host)
            return w
        dist.all_reduce(bucket, op=dist.ReduceOp.SUM, group=group)
    return w


def level_param_ranges(offsets: Dict[str, Tuple[int, Tuple[int, ...]]], levels: int) -> List[Tuple[int, int]]:
    """[first, end) of each level's parameters (enc{l}/*, dec{l}/*) in a ParamStore's offsets; the levels must
    occupy disjoint ranges in level order (VQVAE builds enc0, dec0, enc1, ...)."""
    out = []
    for l in range(levels):
        spans = [(o, o + int(math.prod(sh))) for n, (o, sh) in offsets.items() if n.startswith((f"enc{l}/", f"dec{l}/"))]
        if not spans:
            raise ValueError(f"no parameters of level {l}")
        out.append((min(a for a, _ in spans), max(b for _, b in spans)))
        if l and out[l][0] < out[l - 1][1]:
            raise ValueError(f"level {l}'s parameters interleave with level {l - 1}'s")
    return out


def level_regions(layout: Dict[str, object], grad_ranges: Sequence[Tuple[int, int]]) -> List[List[Tuple[int, int]]]:
    """Per level, the bucket slices its chain alone writes: [its gradient range, its VQ statistics region].
    `grad_ranges` are the levels' parameter ranges in the store; they are widened to a partition of the padded
    gradient region (the alignment gaps between them and the padding at its end, zero on every rank, go with
    the level before them), so the per-level sums cover exactly what the one-bucket exchange covers."""
    P = layout["grads"][1]
    L = len(grad_ranges)
    assert len(layout["stats"]) == L
    starts = [0] + [int(a) for a, _ in grad_ranges[1:]]
    ends = starts[1:] + [P]
    for l, (a, b) in enumerate(grad_ranges):
        if not (starts[l] <= a and b <= ends[l] and a <= b):
            raise ValueError(f"level {l}: parameter range {a}..{b} does not fit {starts[l]}..{ends[l]}")
    return [[(starts[l], ends[l]), tuple(layout["stats"][l])] for l in range(L)]


class _Rccl:
    """ncclAllReduce(SUM, fp32) in place on slices of a device bucket, on the communicator of a torch "nccl" process
    group, queued on the caller's current stream. Capturable: nothing is left for torch's watchdog to poll."""
    FLOAT32, SUM = 7, 0  # ncclFloat32, ncclSum (nccl.h / rccl.h)

    def __init__(self, group, device: torch.device):
        pg = group if group is not None else dist.distributed_c10d._get_default_group()
        be = pg._get_backend(device)
        if not be._comm_ptr():  # communicator created lazily (no device_id at init): one collective creates it
            if torch.cuda.is_current_stream_capturing():
                # a torch-managed collective inside a capture is what the watchdog aborts on (module docstring):
                # build this object before capturing (VQVAE.capture_train_step does)
                raise RuntimeError("vqa_dp: the RCCL communicator does not exist yet and cannot be created while "
                                   "a graph is being captured; call vqa_dp.rccl_direct(group, device) first")
            t = torch.zeros(1, device=device)
            dist.all_reduce(t, group=group)
            torch.cuda.synchronize(device)
        self.be = be  # held: the cache key is this object's identity, which must not be reused while cached
        self.comm = ctypes.c_void_p(be._comm_ptr())
        if not self.comm.value:
            raise RuntimeError("vqa_dp: the process group has no RCCL communicator")
        lib = ctypes.CDLL(loaded_rccl_path())  # the copy torch itself loaded (its communicator lives there)
        self.all_reduce = lib.ncclAllReduce
        self.all_reduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p]
        self.all_reduce.restype = ctypes.c_int
        self.err = lib.ncclGetErrorString
        self.err.argtypes, self.err.restype = [ctypes.c_int], ctypes.c_char_p
        self.log: List[int] = []  # element counts of the collectives issued (tests)

    def current(self) -> bool:
        """Is the cached communicator still the backend's live one? (A destroyed and re-created group, or a
        backend that re-created its communicator, gives another pointer: the entry is rebuilt, never reused.)"""
        try:
            return self.be._comm_ptr() == self.comm.value
        except Exception:
            return False

    def run(self, bucket: torch.Tensor, regions: Sequence[Tuple[int, int]]):
        assert bucket.dtype == torch.float32 and bucket.is_contiguous()
        stream = torch.cuda.current_stream(bucket.device).cuda_stream
        base, sz = bucket.data_ptr(), bucket.element_size()
        for a, b in regions:
            if b <= a:
                continue
            assert 0 <= a and b <= bucket.numel()
            p = base + a * sz
            rc = self.all_reduce(p, p, b - a, self.FLOAT32, self.SUM, self.comm, stream)
            if rc != 0:
                raise RuntimeError(f"ncclAllReduce: {self.err(rc).decode()} ({rc})")
            self.log.append(b - a)


def loaded_rccl_path() -> str:
    """Path of the librccl this process has already mapped (torch's own, or a system RCCL torch links against):
    handing a communicator to a second RCCL instance would be undefined, so no other copy is ever opened."""
    found = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split(None, 5)
                if len(parts) == 6 and os.path.basename(parts[5].strip()).startswith("librccl.so"):
                    found.append(parts[5].strip())
    except OSError:
        pass
    if not found:
        raise RuntimeError("vqa_dp: no librccl is mapped in this process (is the process group's backend RCCL?)")
    return found[0]


_RCCL: Dict[Tuple[int, str], _Rccl] = {}


def rccl_direct(group, device: torch.device) -> _Rccl:
    """The direct-RCCL issuer of `group` on `device`, keyed on the identity of the group's backend object and
    checked against its live communicator pointer at every call (see `_Rccl.current`)."""
    pg = group if group is not None else dist.distributed_c10d._get_default_group()
    be = pg._get_backend(device)
    key = (id(be), str(device))
    ent = _RCCL.get(key)
    if ent is None or ent.be is not be or not ent.current():
        ent = _RCCL[key] = _Rccl(group, device)
    return ent


def reset():
    """Forget every cached communicator (call before `dist.destroy_process_group()`)."""
    _RCCL.clear()


def exchange_regions(bucket: torch.Tensor, regions: Sequence[Tuple[int, int]], group=None) -> int:
    """Sum each slice bucket[a:b] over ranks (no-op on one rank): on RCCL one ncclAllReduce per slice issued
    directly (`_Rccl`, capturable), on gloo `exchange` per slice (host-staged)."""
    w = world_size(group)
    if not active(group):
        return w
    if bucket.is_cuda and device_side(group):
        rccl_direct(group, bucket.device).run(bucket, regions)
        return w
    for a, b in regions:
        if b > a:
            exchange(bucket[a:b], group)
    return w


def global_row_range(n_local: int, group=None):
    """(row_offset, N_global) of this rank's VQ rows in the global flattened batch."""
    return rank(group) * n_local, world_size(group) * n_local
