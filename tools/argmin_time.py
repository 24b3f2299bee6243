"""Time vqa_vq_argmin_split (bf16 z, exact 3-plane codebook) at the cfg2 levels' row counts (GPU dev tool).

    python tools/argmin_time.py [N ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402

import vqa_lib as V  # noqa: E402

dev = torch.device("cuda", 0)
D, K = 64, 2048
g = torch.Generator(device=dev).manual_seed(0)
E = torch.randn(D, K, device=dev, generator=g) * 0.05
esq = torch.empty(K, device=dev)
V.vq_sqnorm(E, esq)
E3 = torch.empty(K, 3, D, dtype=torch.bfloat16, device=dev)
V.vq_split_bf16x3(E, E3)
for N in [int(a) for a in sys.argv[1:]] or (262144, 131072, 65536, 32768, 8192):
    z = torch.randn(N, D, device=dev, generator=g).to(torch.bfloat16)
    idx = torch.empty(N, dtype=torch.int64, device=dev)
    f = lambda: V.vq_argmin_split(z, E3, esq, idx)  # noqa: E731
    f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    s.record()
    for _ in range(reps):
        f()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / reps
    tf = 2.0 * N * K * D * 3 / (us * 1e-6) / 1e12
    print(f"N={N:7d} K={K} D={D}: {us:8.1f} us  {tf:7.1f} TFLOP/s (3 bf16 planes)")
