"""Run the fused residual-block kernels on one shape a few times (GPU dev tool, for rocprofv3 --pmc passes).

    python tools/resblock_one.py [fwd|bwd|both] [T] [dilation] [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402

import vqa_lib as V  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "both"
T = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
d = int(sys.argv[3]) if len(sys.argv) > 3 else 9
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
B, C = 32, 32
dev = torch.device("cuda", 0)
x = torch.randn(B, T, C, device=dev).to(torch.bfloat16)
dy = torch.randn(B, T, C, device=dev).to(torch.bfloat16)
wa, wb = torch.randn(3, C, C, device=dev) * 0.1, torch.randn(3, C, C, device=dev) * 0.1
ba, bb = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
y, dx = torch.empty_like(x), torch.empty_like(x)
gw = [torch.empty(3, C, C, device=dev), torch.empty(C, device=dev)] * 2
for _ in range(reps):
    if which in ("fwd", "both"):
        V.resblock_fwd(x, wa, ba, wb, bb, y, d)
    if which in ("bwd", "both"):
        V.resblock_bwd(dy, x, wa, ba, wb, bb, dx, *gw, d)
torch.cuda.synchronize()
print("ok")
