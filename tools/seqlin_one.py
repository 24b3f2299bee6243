"""Run one sequence-linear shape repeatedly (GPU dev tool for PMC passes): python tools/seqlin_one.py K N TAPS [prep]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]
import torch  # noqa: E402
import vqa_lib as V  # noqa: E402

K, N, taps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
prep = len(sys.argv) > 4 and sys.argv[4] == "prep"
dev = torch.device("cuda:0")
x = torch.randn(8, 8192, K, device=dev).bfloat16()
r = torch.randn(8, 8192, N, device=dev).bfloat16()
y = torch.empty_like(r)
w = torch.randn(taps, K, N, device=dev) * 0.05
b = torch.zeros(N, device=dev)
wp = torch.empty(taps, N, K, dtype=torch.bfloat16, device=dev)
V.seqlin_prep([(w, wp, taps, K, N, False)], torch.bfloat16)
for _ in range(10):
    if prep:
        V.seqlin_fwd_prepped(x, wp, b, y, 8192, taps=taps, residual=r)
    else:
        V.seqlin_fwd(x, w if taps == 3 else w[0], b, y, 8192, taps=taps, residual=r)
torch.cuda.synchronize()
