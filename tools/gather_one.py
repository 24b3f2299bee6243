"""Run the decoder's 32 -> 32 Conv1DTranspose (k4, stride 2; PAIR-mode gather_mfma_kernel) at the cfg2
level-0 shape a few times (GPU dev tool, for rocprofv3 passes and timing).

    python tools/gather_one.py [T_in] [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402

import vqa_lib as V  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
B, C = 32, 32
dev = torch.device("cuda", 0)
x = torch.randn(B, T, C, device=dev).to(torch.bfloat16)
w = torch.randn(4, C, C, device=dev) * 0.1
b = torch.zeros(C, device=dev)
y = torch.empty(B, 2 * T, C, device=dev, dtype=torch.bfloat16)
f = lambda: V.conv1d_transpose_fwd(x, w, b, None, y, B, T, 2 * T, C, C, 4, 2, 1, 0, V.BF16)
f()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(reps):
    f()
e.record()
torch.cuda.synchronize()
us = s.elapsed_time(e) * 1e3 / reps
mb = (x.numel() + y.numel()) * 2 / 1e6
print(f"T_in={T} convT 32->32: {us:.1f} us, {mb:.1f} MB, {mb / us * 1e-3 * 1e3:.0f} GB/s")
