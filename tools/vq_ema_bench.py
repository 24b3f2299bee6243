"""Time vqa_vq_quantize with the EMA sums (GPU dev tool): one hot code vs uniform codes, per N.

    python tools/vq_ema_bench.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402

import vqa_lib as V  # noqa: E402

dev = torch.device("cuda", 0)
D, K = 64, 2048
for N in (16384, 65536, 262144):
    z = torch.randn(N, D, device=dev).to(torch.bfloat16)
    ET = torch.randn(K, D, device=dev)
    for name, idx in (("hot", torch.zeros(N, dtype=torch.int64, device=dev)),
                      ("uniform", torch.randint(0, K, (N,), device=dev))):
        q = torch.empty_like(z)
        commit = torch.empty(1, device=dev)
        ms = torch.zeros(K, D, device=dev)
        ns = torch.zeros(K, device=dev)
        for with_ema in (False, True):
            f = lambda: V.vq_quantize(z, ET, idx, q, commit, ms if with_ema else None, ns if with_ema else None, 0.25)
            f()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                f()
            e.record()
            torch.cuda.synchronize()
            print(f"N={N:7d} {name:8s} ema={with_ema!s:5s} {s.elapsed_time(e) / 20 * 1000:8.1f} us", flush=True)
