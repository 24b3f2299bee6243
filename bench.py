"""bench.py — VQ-VAE train-step throughput on MI355X (BASELINE.json metric), one process per GPU.

Workload (BASELINE config 2, "SMALL_VQ_VAE 3-level"): levels 3, latent 64, codebook 2048, down_depth
[3,2,2], strides [2,2,2] (hops 8/32/128), residual width 32, depth 4, dilation factor 3; 65,536-frame
44.1 kHz synthetic chunks, batch 32 per GPU, bf16 activations with fp32 weights / VQ state / Adam.
A step = one full VQVAE.train_step (forward, spectral + MSE + commitment losses, backward, Keras Adam,
codebook EMA with dead-code reset), replayed from a hipGraph. N > 1: data parallel (weak scaling), one
RCCL all_reduce of [grads | EMA sums | reset rows | losses] per step. `--gpus N` is authoritative: a bare
`python bench.py --gpus N` starts the N ranks itself (a child `torch.distributed.run`, 127.0.0.1 rendezvous);
under a launcher each rank refuses to run unless WORLD_SIZE == N.

Prints ONE JSON line on rank 0. Also reports:
  roofline     — the dominant kernel (fused residual-block backward) — its algorithmic bytes (SURVEY §8d layer
                 model) / its average duration: its launches of one step are recorded after the timed region
                 and timed back to back in hipGraphs with HIP events on the stream it runs on; `traffic` =
                 HBM bytes per launch from profiles/pmc_traffic.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE,
                 gfx950 correction) when present; compulsory_* = the 3 tensors the fused kernel must move;
  cpu_baseline — the oracle (torch-CPU fp32 restatement of the reference op sequence) timed on the host
                 cores on a bounded sample (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "vae-based-music--deep-generative-models_amd")
sys.path[:0] = [PKG, ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "audio-samples/sec/GPU VQ-VAE train step, 44.1kHz 65536-frame chunks @1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
BF16_DENSE_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA peak (no sparsity)
CFG2 = dict(levels=3, latent_dim=64, down_depth=[3, 2, 2], strides=[2, 2, 2], num_embeddings=2048,
            residual_width=32, residual_depth=4, dilation_factor=3)
DOMINANT = "resblock_bwd_kernel<bf16>"  # fused residual-block backward (h recomputed): 120 launches per step


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--batch", type=int, default=32, help="per-GPU batch")
    p.add_argument("--seq", type=int, default=65536)
    p.add_argument("--dtype", default="bf16")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-roofline", action="store_true", help="skip the roofline replays (PMC passes)")
    p.add_argument("--cpu-batch", type=int, default=8)
    p.add_argument("--cpu-steps", type=int, default=4)
    p.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    p.add_argument("--no-prior", action="store_true", help="skip the config-4 / config-5 legs")
    p.add_argument("--prior-batch", type=int, default=8, help="config-4 leg: sequences per GPU")
    p.add_argument("--prior-steps", type=int, default=10)
    p.add_argument("--decode-samples", type=int, default=16)
    p.add_argument("--decode-len", type=int, default=1024)
    p.add_argument("--no-fp32", action="store_true", help="skip the fp32 config-2 leg")
    p.add_argument("--fp32-steps", type=int, default=5)
    return p.parse_args()


class KernelTimer:
    """Roofline of the dominant kernel, resblock_bwd_kernel<bf16> (resnet.py:7-29 backward, one launch per
    residual block): record every vqa_resblock_bwd call of one step (in order, with its own tensors), then
    capture ALL of them back to back into one hipGraph and time its replays with HIP events on the stream
    libvqa launches on. One graph for the whole mix amortises the graph-launch overhead over the step's
    launches, so the per-launch average is the kernels' own duration (plus the ~1 us inter-kernel gap of a
    graph) and matches rocprofv3's average for the kernel. The weight-gradient partial reduction is left
    out (its own kernel).

    Algorithmic bytes per launch (SURVEY.md §8d layer model): the launch does the data- and
    weight-gradient of the block's two convs, 2 x (|in| + |out|) per conv = 8 activation tensors of
    B*T*32 elements. Compulsory bytes (what the fused kernel must move: dy, x read, dx written) = 3."""

    def __init__(self, V):
        self.V = V
        self.calls = []
        self.rows = []
        self.orig = None

    def flops_per_step(self) -> float:
        """Algorithmic MFMA flops of the step's launches: five k=3, 32->32 convs (h recompute, dW_b, dh, dx,
        dW_a), 2*3*32*32 flop per row each, over the B*T rows (the halo recompute is not counted)."""
        return float(sum(5 * 2 * 3 * 32 * 32 * B * T for B, T, _ in self.rows))

    def __enter__(self):
        self.orig = f = self.V.resblock_bwd

        def wrapped(dy, x, *rest, _f=f):
            unit = x.numel() * x.element_size()
            self.calls.append(((dy, x) + tuple(rest), 8 * unit, 3 * unit))
            self.rows.append((x.shape[0], x.shape[1], rest[-2]))  # (B, T, dilation)
            return _f(dy, x, *rest)
        self.V.resblock_bwd = wrapped
        return self

    def __exit__(self, *a):
        self.V.resblock_bwd = self.orig

    def measure(self, reps=5):
        """-> (launches per step, total us per step, algorithmic bytes per step, compulsory bytes per step)."""
        if not self.calls:
            return 0, 0.0, 0, 0
        stream = torch.cuda.current_stream()
        f = self.orig
        deferred = self.V.Deferred()  # partials left unreduced: time the kernel alone
        runs = [args[:-1] + (deferred,) for args, _, _ in self.calls]
        for args in runs:
            f(*args)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for args in runs:
                f(*args)
        g.replay()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        for _ in range(reps):
            g.replay()
        e.record(stream)
        torch.cuda.synchronize()
        n = len(runs)
        us_total = s.elapsed_time(e) * 1e3 / reps
        return n, us_total, sum(c[1] for c in self.calls), sum(c[2] for c in self.calls)


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def cpu_baseline(batch, steps, seq):
    """The oracle (reference op sequence, fp32) on the host cores this process may use: every CPU of its
    affinity mask, capped by OMP_NUM_THREADS when the box sets its CPU share that way (16 per GPU)."""
    from oracle import vqvae_ref as R
    allowed = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(allowed, omp) if omp > 0 else allowed
    torch.set_num_threads(threads)
    cfg = R.RefConfig(input_len=seq, **CFG2)
    m = R.RefVQVAE(cfg, R.init_params(cfg, 1), R.init_vq_state(cfg, 2), dtype=torch.float32)
    x = R.synthetic_batch(batch, seq, seed=999)
    m.train_step(x)  # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        m.train_step(x)
    dt = time.perf_counter() - t0
    return {"value": batch * seq * steps / dt, "unit": "audio-samples/s", "cores": threads, "kind": "port",
            "cpu": _cpu_model(), "nproc": os.cpu_count(), "affinity_cpus": allowed,
            "sample": f"oracle torch-CPU fp32 train step (dense one-hot GEMMs, N x K distances, TF-style STFT) on "
                      f"the cfg2 architecture, {batch} x {seq}-frame chunks, {steps} timed steps after 1 warm-up, "
                      f"{threads} threads of {_cpu_model()} (nproc {os.cpu_count()}, {allowed} in this process's "
                      f"affinity mask, OMP_NUM_THREADS {omp or 'unset'}; {dt:.1f} s)",
            "cores_note": "the GPU box gives one GPU's job a CPU share of 16 threads and sets OMP_NUM_THREADS=16 to "
                          "say so (its rules: leave that setting and size thread pools to the share); every CPU of "
                          "the affinity mask is used where no such share is set"}


def fp32_leg(a, dev, world, batches):
    """Config 2 at the reference's own arithmetic precision (fp32 activations, the exact fp32 MFMA path), beside the
    bf16 headline: the same architecture, batch, chunk length, graph replay and clock as the main line (an extra key;
    `value` stays bf16 config 2, the dtype BASELINE.json names)."""
    from vqvae import VQVAE
    m = VQVAE((a.seq, 1), dtype="fp32", device=dev, **CFG2)
    m.compile()
    m.capture_train_step(batches[0], warmup=1)
    m.train_step(batches[1])
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(a.fp32_steps):
        m.train_step(batches[i % len(batches)])
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    el = time.perf_counter() - t0
    if dist.is_initialized():
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    v = a.batch * a.seq * a.fp32_steps * world / el
    out = {"metric": METRIC + " (fp32)", "value": round(v, 1), "value_per_gpu": round(v / world, 1),
           "unit": "audio-samples/s", "n_gpus": world, "steps": a.fp32_steps,
           "ms_per_step": round(el / a.fp32_steps * 1e3, 3), "dtype": "fp32",
           "config": {"workload": "BASELINE config 2 in fp32 (the reference's arithmetic)", "global_batch": a.batch * world,
                      "seq_len": a.seq, "graph": True},
           "final_loss": round(float(m.results()["loss"]), 5)}
    del m
    torch.cuda.empty_cache()
    return out


def prior_legs(a, dev, world, rank):
    """BASELINE configs 4 and 5 beside the config-2 line (extra keys; `value` stays config 2's):
      config4_prior_train: SMALL_PRIOR (width 128, depth 6, 2 heads, 4 blocks, 2048 bins) Prior.train_step over
        ctx = 8192 top-level codes, `prior_batch` sequences per GPU, bf16, the whole step (both teacher-forcing
        passes, backward, Keras Adam) replayed from a hipGraph; under DP two graphs around the one all_reduce of
        the prior's bucket (weak scaling, the same barrier + max-over-ranks clock as the main line);
      config5_upsampler_decode (rank 0, N = 1): the SMALL_UPSAMPLER form (the same transformer conditioned on the
        level above through ConditionerNet) drawing `decode_samples` samples x `decode_len` positions by ancestral
        sampling, one persistent decode launch per window (prior.py:374-408, Sampler.py:72-109).
    Synthetic uniform codes, random-init weights (prior.py:240-335)."""
    from prior import FMHABasedAutoregressiveModel, Prior
    kw = dict(width=128, depth=6, heads=2, blocks=4, attn_stacks=1, drop_out_rate=0.0)
    ctx, bins = 8192, 2048
    out = {}
    pr = Prior(2, [(ctx * 16,), (ctx * 4,), (ctx,)], bins, [3, 2, 2], [2, 2, 2], None, kw, None, dtype=a.dtype,
               device=dev)  # under DP the default process group (vqa_dp)
    g = torch.Generator(device=dev).manual_seed(11 + rank)
    codes = torch.randint(0, bins - 1, (a.prior_batch, ctx), device=dev, generator=g)
    pr.capture_train_step(codes, warmup=1)
    pr.train_step(codes)  # the first replay uploads the graph
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.prior_steps):
        pr.train_step(codes)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    el = time.perf_counter() - t0
    if dist.is_initialized():
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    tok = a.prior_batch * ctx * a.prior_steps * world / el
    out["config4_prior_train"] = {
        "metric": "tokens/s prior train step (SMALL_PRIOR, ctx 8192), whole job", "value": round(tok, 1),
        "value_per_gpu": round(tok / world, 1), "unit": "tokens/s", "n_gpus": world, "steps": a.prior_steps,
        "ms_per_step": round(el / a.prior_steps * 1e3, 3), "dtype": a.dtype, "scaling": "weak",
        "config": {"workload": "BASELINE config 4", "batch_per_gpu": a.prior_batch, "ctx": ctx, "bins": bins,
                   "parallelism": f"dp{world}", "graph": True, **kw},
        "loss": round(float(pr.results()["loss"]), 5)}
    del pr
    torch.cuda.empty_cache()
    if world == 1 and rank == 0:
        m = FMHABasedAutoregressiveModel(bins, 128, 6, 4, heads=2, attn_stacks=1, drop_out_rate=0.0,
                                         context_length=(ctx,), level=0, levels=2, zq_shapes=[(ctx,), (ctx // 4,)],
                                         downs=[3, 2], strides=[2, 2],
                                         cond_kwargs=dict(dilation_factor=3, dilation_cycle=4, residual_width=32,
                                                          residual_depth=8), dtype="fp32", device=dev)
        g = torch.Generator(device=dev).manual_seed(2)
        up = torch.randint(0, bins - 1, (a.decode_samples, ctx // 4), device=dev, generator=g)
        m.sample(a.decode_samples, max_length=16, x_cond=up, seed=1)  # warm-up: conditioner + decode kernels
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        toks = m.sample(a.decode_samples, max_length=a.decode_len, x_cond=up, seed=2)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        out["config5_upsampler_decode"] = {
            "metric": "tokens/s ancestral decode (upsampler prior + ConditionerNet)",
            "value": round(a.decode_samples * a.decode_len / el, 1), "unit": "tokens/s", "n_gpus": 1,
            "ms_per_position": round(el / a.decode_len * 1e3, 4), "samples": a.decode_samples,
            "positions": a.decode_len, "dtype": "fp32 (decode)",
            "config": {"workload": "BASELINE config 5 (one window, conditioner included)", "ctx": ctx, "bins": bins,
                       **kw},
            "tokens_in_range": bool(((toks >= 0) & (toks < bins)).all())}
        del m
        torch.cuda.empty_cache()
    return out


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a) -> int:
    """`--gpus N` with N > 1 and no WORLD_SIZE in the environment: this process is only the launcher. It starts
    `python -m torch.distributed.run --nproc-per-node N ... bench.py <same arguments>` as a CHILD process (one rank
    per GPU, rendezvous on 127.0.0.1) and returns its exit code. Nothing here touches the GPU (counting devices
    does not initialise it), and nothing execs: the ranks are children, the launcher waits."""
    import subprocess
    backend = os.environ.get("VQA_DIST_BACKEND", "nccl")
    if backend == "nccl":
        have = torch.cuda.device_count()
        if have < a.gpus:
            print(f"bench.py: --gpus {a.gpus} needs {a.gpus} visible GPUs for RCCL, {have} visible", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.call(cmd, env=env)


def main():
    a = parse()
    if a.gpus < 1:
        print(f"bench.py: --gpus must be >= 1 (got {a.gpus})", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch_ranks(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        # the rank count comes from the launcher; --gpus must name the same number or the line would mislabel
        print(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}; run `bench.py --gpus N` (it starts the N ranks "
              f"itself) or a launcher with --nproc-per-node equal to --gpus", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # VQA_DIST_BACKEND=gloo + ranks sharing one GPU (local rank wrapped onto the visible devices) rehearses the
    # DP path (split graphs around the exchange) on a one-GPU box; the driver's N>1 runs use RCCL ("nccl")
    backend = os.environ.get("VQA_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local %= max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # VQA_DP_FORCE=1 (rehearsal, tests/test_gpu_rccl.py): the DP branch — process group, the exchange's collective
    # on the device bucket, split graphs — at N = 1 too (torchrun --nproc-per-node 1), so RCCL runs on one GPU
    force = os.environ.get("VQA_DP_FORCE") == "1"
    if world > 1 or force:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        if force:
            import vqa_dp
            vqa_dp.FORCE_COLLECTIVE = True
    import vqa_lib as V
    from data_utils import synthetic_batch_device
    from vqvae import VQVAE

    model = VQVAE((a.seq, 1), dtype=a.dtype, device=dev, **CFG2)
    model.compile()
    # the device feed: 4 batches generated in HBM by vqa_synthetic_batch (seeded per rank)
    batches = [synthetic_batch_device(a.batch, a.seq, seed=1234 + 7919 * i, rank=rank, device=dev) for i in range(4)]
    if not a.no_graph:
        # 1 eager step (FFT plans, LDS limits), capture, then warmup-1 untimed replays: the first replays
        # of a fresh hipGraph carry its upload cost
        model.capture_train_step(batches[0], warmup=1)
        for i in range(max(a.warmup - 1, 1)):
            model.train_step(batches[i % 4])
    else:
        for i in range(a.warmup):
            model.train_step(batches[i % 4])
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(a.steps):
        model.train_step(batches[i % 4])
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist.is_initialized():
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    loss = float(model.results()["loss"])

    # roofline: record the dominant kernel's launches of one step, then time them back to back
    with KernelTimer(V) as kt:
        model._compute(batches[0], True)
    torch.cuda.synchronize()
    n_launch, us_total, nbytes, cbytes = (0, 0.0, 0, 0) if a.no_roofline else kt.measure()
    achieved = nbytes / (us_total * 1e-6) / 1e9 if us_total > 0 else 0.0
    compulsory = cbytes / (us_total * 1e-6) / 1e9 if us_total > 0 else 0.0
    pmc = {}
    if os.path.exists(a.pmc_json):
        try:
            pmc = json.load(open(a.pmc_json))
        except Exception:
            pmc = {}
    traffic = pmc.get("per_launch_bytes")
    # provenance of the counter file: a traffic figure read from another library build is flagged stale
    lib_sha = None
    try:
        import hashlib
        lib_sha = hashlib.sha256(open(V.LIB_PATH, "rb").read()).hexdigest()
    except Exception:
        pass
    avg_us = us_total / max(n_launch, 1)
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": DOMINANT,
            "launches_per_step": n_launch, "avg_launch_us": round(avg_us, 2),
            "algorithmic_bytes_per_launch": int(nbytes / max(n_launch, 1)),
            "compulsory_bytes_per_launch": int(cbytes / max(n_launch, 1)),
            "compulsory_GBps": round(compulsory, 1), "compulsory_frac": round(compulsory / HBM_PEAK_GBS, 4),
            "kernel_ms_per_step": round(us_total / 1e3, 3),
            "traffic_source": {"file": os.path.relpath(a.pmc_json, ROOT) if pmc else None,
                               "commit": pmc.get("commit"), "measured_utc": pmc.get("measured_utc"),
                               "lib_sha256": pmc.get("lib_sha256"), "loaded_lib_sha256": lib_sha,
                               "same_library": bool(lib_sha and pmc.get("lib_sha256") == lib_sha)}}
    if traffic and avg_us > 0:
        # measured HBM bytes (PMC, profiles/) over the live average launch time: the real bandwidth fraction
        roof["traffic_GBps"] = round(traffic / (avg_us * 1e-6) / 1e9, 1)
        roof["traffic_frac"] = round(traffic / (avg_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
    if n_launch:
        # MFMA: the launch's matrix flops (5 k=3 convs over the tile rows incl. the recomputed halo) against
        # the dense bf16 peak, and the PMC busy fraction (SQ_VALU_MFMA_BUSY_CYCLES) when measured
        fl = kt.flops_per_step()
        roof["mfma"] = {"tflops": round(fl / (us_total * 1e-6) / 1e12, 1), "peak_tflops": BF16_DENSE_TFLOPS,
                        "frac": round(fl / (us_total * 1e-6) / 1e12 / BF16_DENSE_TFLOPS, 4),
                        "busy_frac_pmc": pmc.get("mfma_busy_frac")}

    legs = {}
    if not a.no_fp32 and a.dtype == "bf16":
        try:
            legs["config2_fp32"] = fp32_leg(a, dev, world, batches)
        except Exception as e:  # an extra leg must never cost the config-2 line
            legs["config2_fp32"] = {"error": f"{type(e).__name__}: {e}"[:400]}
    if not a.no_prior:
        try:
            legs.update(prior_legs(a, dev, world, rank))
        except Exception as e:  # an extra leg must never cost the config-2 line
            legs["prior_legs_error"] = f"{type(e).__name__}: {e}"[:400]

    out = None
    if rank == 0:
        cpu = None
        if world == 1 and not a.no_cpu_baseline:
            cpu = cpu_baseline(a.cpu_batch, a.cpu_steps, a.seq)
        # value: the whole job's audio-samples/s (all ranks; the driver derives scaling from it);
        # value_per_gpu: the metric's per-GPU reading (B_per_gpu * T * steps / wall-seconds)
        value = a.batch * a.seq * a.steps * world / elapsed
        out = {"metric": METRIC, "value": round(value, 1), "value_per_gpu": round(value / world, 1),
               "value_is": "whole-job aggregate over n_gpus (the bench contract: total audio-samples/s of all ranks); "
                           "value_per_gpu is the metric's per-GPU reading",
               "unit": "audio-samples/s", "n_gpus": world,
               "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": a.dtype,
               "data": "synthetic 44.1 kHz sine+noise chunks (SURVEY.md §8d) generated on the device "
                       "(vqa_synthetic_batch), random-init weights",
               "config": {"workload": "SMALL_VQ_VAE 3-level VQ-VAE train step (BASELINE config 2)",
                          "model": "VQVAE levels=3 latent=64 K=2048 down_depth=[3,2,2] width=32 depth=4 dil=3",
                          "global_batch": a.batch * world, "seq_len": a.seq, "parallelism": f"dp{world}",
                          "graph": not a.no_graph, "final_loss": round(loss, 5),
                          "exchange": ("per-level, overlapped" if model.overlap_exchange else "one bucket after the join")
                          if dist.is_initialized() else None},
               "roofline": roof, "cpu_baseline": cpu, **legs}
        if dist.is_initialized() and model.overlap_exchange:
            out["config"]["exchange_note"] = ("VQA_DP_OVERLAP=1 forced the per-level exchange on; its captured "
                                              "multi-rank form had not run on hardware before this line (DESIGN.md §5)")
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.barrier()
        import vqa_dp
        vqa_dp.reset()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
