"""Prior measurements (BASELINE configs 4 and 5) on one MI355X: prints one JSON line per workload.

  train : SMALL_PRIOR (width 128, depth 6, heads 2, blocks 4, row/col/prev-row, bins 2048) Prior.train_step over
          ctx = 8192 top-level codes, bf16 activations, the whole step (two teacher-forcing passes, backward, Adam)
          replayed from a hipGraph; tokens/s = B * ctx * steps / seconds.
  sample: SMALL_UPSAMPLER-style ancestral decode (the same transformer conditioned on upper-level codes through
          ConditionerNet) — one persistent decode launch for N samples x L positions; tokens/s.
Synthetic codes (uniform over the codebook), random-init weights. The cpu leg times the oracle's train step
(oracle/prior_ref.py, torch CPU fp32) on a bounded sample.
    python tools/bench_prior.py [--batch 8] [--steps 10] [--samples 16] [--sample-len 2048] [--no-cpu]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--ctx", type=int, default=8192)
    ap.add_argument("--bins", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--samples", type=int, default=16)
    ap.add_argument("--sample-len", type=int, default=2048)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    from prior import Prior, FMHABasedAutoregressiveModel
    kw = dict(width=128, depth=6, heads=2, blocks=4, attn_stacks=1, drop_out_rate=0.0)
    dev = torch.device("cuda:0")
    if a.only in ("", "train"):
        pr = Prior(2, [(a.ctx * 16,), (a.ctx * 4,), (a.ctx,)], a.bins, [3, 2, 2], [2, 2, 2], None, kw, None,
                   dtype=a.dtype, device="cuda")
        g = torch.Generator(device=dev).manual_seed(1)
        codes = torch.randint(0, a.bins - 1, (a.batch, a.ctx), device=dev, generator=g)
        pr.capture_train_step(codes, warmup=a.warmup)
        pr.train_step(codes)  # first replay uploads the graph
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            pr.train_step(codes)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        tok = a.batch * a.ctx * a.steps / el
        out = {"metric": "tokens/sec/GPU prior train step (SMALL_PRIOR, ctx 8192)", "value": round(tok, 1),
               "unit": "tokens/s", "n_gpus": 1, "steps": a.steps, "ms_per_step": round(el / a.steps * 1e3, 3),
               "dtype": a.dtype, "data": "synthetic uniform codes, random-init weights",
               "config": {"workload": "BASELINE config 4 (per GPU)", "batch": a.batch, "ctx": a.ctx, "bins": a.bins,
                          **kw}, "loss": float(pr.results()["loss"])}
        # kernel-level rooflines of the step's dominant pieces, timed as hipGraph replays (HIP events on the
        # launching stream): the sequence-linear layer (HBM-bound: bytes = X + Y + residual), the row
        # attention forward and the fused head (MFMA work, exp-heavy)
        import vqa_lib as V
        M = a.batch * a.ctx
        cdt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
        esz = 2 if a.dtype == "bf16" else 4
        x = torch.randn(a.batch, a.ctx, 128, device=dev).to(cdt)
        r = torch.randn_like(x)
        y = torch.empty_like(x)
        w = torch.randn(128, 128, device=dev) * 0.05
        bb = torch.zeros(128, device=dev)
        q = torch.randn(a.batch, a.ctx, 32, device=dev).to(cdt)
        o = torch.empty_like(q)
        lse = torch.empty(a.batch, a.ctx, 2, device=dev)
        wt = torch.empty(a.bins, 128, dtype=cdt, device=dev)
        V.head_wt(torch.randn(128, a.bins, device=dev) * 0.05, wt)
        hb = torch.zeros(a.bins, device=dev)
        hl = torch.empty(M, device=dev)
        am = torch.empty(M, dtype=torch.int64, device=dev)

        def timed(fn, reps=20):
            fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(reps):
                    fn()
            g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / reps * 1e3  # us

        wp = torch.empty(1, 128, 128, dtype=cdt, device=dev)
        V.seqlin_prep([(w, wp, 1, 128, 128, False)], cdt)
        t_lin = timed(lambda: V.seqlin_fwd_prepped(x, wp, bb, y, a.ctx, residual=r))
        lin_bytes = 3 * M * 128 * esz
        t_att = timed(lambda: V.attn_fwd(q, q, q, o, lse, 0, a.ctx // 4, 2, 0.25))
        att_flop = a.batch * 2 * 4 * (a.ctx // 4) * (a.ctx // 4 + 64) / 2 * 16 * 2 * 2
        t_head = timed(lambda: V.head_fwd(x, wt, hb, hl, amax=am))
        head_flop = 2.0 * M * 128 * a.bins
        out["roofline"] = {"kernel": "seqlin_d_kernel<bf16,128,1,8,8> (Dense 128->128 + residual, the mlp form, prepared weights)",
                           "bound": "hbm", "achieved": round(lin_bytes / t_lin / 1e3, 1), "peak": 8000.0,
                           "unit": "GB/s", "frac": round(lin_bytes / t_lin / 1e3 / 8000.0, 4),
                           "avg_launch_us": round(t_lin, 2), "algorithmic_bytes_per_launch": lin_bytes}
        out["kernels"] = {
            "attn_fwd_row": {"us": round(t_att, 1), "tflops": round(att_flop / t_att / 1e6, 1),
                             "mfma_frac": round(att_flop / t_att / 1e6 / 2500.0, 4)},
            "head_fwd": {"us": round(t_head, 1), "tflops": round(head_flop / t_head / 1e6, 1),
                         "mfma_frac": round(head_flop / t_head / 1e6 / 2500.0, 4)}}
        if not a.no_cpu:
            import numpy as np
            from oracle import prior_ref as P
            torch.set_num_threads(min(16, os.cpu_count() or 1))
            cfg = P.PriorConfig(bins=a.bins, ctx=a.ctx, width=128, depth=6, heads=2, blocks=4, attn_stacks=1)
            p = P.to_torch(P.init_params(cfg, 1), torch.float32)
            c = torch.randint(0, a.bins - 1, (1, a.ctx))
            m = torch.zeros(1, a.ctx, dtype=torch.bool)
            t0 = time.perf_counter()
            P.train_step_grads(p, cfg, c, m)
            ce = time.perf_counter() - t0
            out["cpu_baseline"] = {"value": round(a.ctx / ce, 1), "unit": "tokens/s", "cores": torch.get_num_threads(),
                                   "kind": "port", "sample": f"oracle torch-CPU fp32 train step (both passes + "
                                   f"autograd), 1 x {a.ctx} tokens, {ce:.1f} s"}
        print(json.dumps(out), flush=True)
        del pr
        torch.cuda.empty_cache()
    if a.only in ("", "sample"):
        m = FMHABasedAutoregressiveModel(a.bins, 128, 6, 4, heads=2, attn_stacks=1, drop_out_rate=0.0,
                                         context_length=(a.ctx,), level=0, levels=2, zq_shapes=[(a.ctx,), (a.ctx // 4,)],
                                         downs=[3, 2], strides=[2, 2],
                                         cond_kwargs=dict(dilation_factor=3, dilation_cycle=4, residual_width=32,
                                                          residual_depth=8), dtype="fp32", device="cuda")
        g = torch.Generator(device=dev).manual_seed(2)
        up = torch.randint(0, a.bins - 1, (a.samples, a.ctx // 4), device=dev, generator=g)
        m.sample(a.samples, max_length=16, x_cond=up, seed=1)  # warm-up (conditioner + decode)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out_tok = m.sample(a.samples, max_length=a.sample_len, x_cond=up, seed=2)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(json.dumps({"metric": "tokens/sec ancestral decode (upsampler prior + ConditionerNet)",
                          "value": round(a.samples * a.sample_len / el, 1), "unit": "tokens/s", "n_gpus": 1,
                          "ms_per_position": round(el / a.sample_len * 1e3, 4), "samples": a.samples,
                          "positions": a.sample_len, "dtype": "fp32 (decode)",
                          "config": {"workload": "BASELINE config 5", "ctx": a.ctx, "bins": a.bins, **kw},
                          "tokens_in_range": bool(((out_tok >= 0) & (out_tok < a.bins)).all())}), flush=True)

    if a.only in ("", "sampler"):
        # Sampler.py end to end: three levels top-down (n_ctxs of Sampler.py:127, the SMALL_* prior / conditioner
        # settings of :24-25), each window one persistent decode launch, the lower ones conditioned on the codes
        # drawn above them through ConditionerNet
        from sampler import VQVAESampler
        n_ctxs = [8192, 8192, 6144]
        s = VQVAESampler([3, 2, 2], [2, 2, 2], n_ctxs, codebook_size=a.bins, dtype="fp32", device="cuda")
        VQVAESampler([3, 2, 2], [2, 2, 2], [64, 16, 4], codebook_size=a.bins, priors=None, dtype="fp32",
                     device="cuda").sample(a.samples, seed=1)  # warm-up (every kernel, conditioner included)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        zs = s.sample(a.samples, seed=2)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        ntok = a.samples * sum(n_ctxs)
        print(json.dumps({"metric": "tokens/sec VQVAESampler 3-level ancestral sampling (Sampler.py)",
                          "value": round(ntok / el, 1), "unit": "tokens/s", "n_gpus": 1, "seconds": round(el, 3),
                          "samples": a.samples, "n_ctxs": n_ctxs, "dtype": "fp32 (decode)",
                          "config": {"workload": "BASELINE config 5 (Sampler.py)", "bins": a.bins, **kw},
                          "shapes": [list(z.shape) for z in zs],
                          "tokens_in_range": bool(all(((z >= 0) & (z < a.bins)).all() for z in zs))}), flush=True)


if __name__ == "__main__":
    main()
