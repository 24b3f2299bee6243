"""Run the spectral loss kernels on the cfg2 shape a few times (GPU dev tool, for rocprofv3 --pmc passes and
quick timing): the target spectrograms once, then the loss + gradient of a reconstruction.

    python tools/spec_one.py [reps] [--time]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402

from data_utils import SpectralTarget, multispectral_loss_and_grad, synthetic_batch_device  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 3
x = synthetic_batch_device(32, 65536, seed=1)
r = x + 0.01 * torch.randn_like(x)
for _ in range(2):
    t = SpectralTarget(x)
    multispectral_loss_and_grad(t, r)
torch.cuda.synchronize()
if "--time" in sys.argv:
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        t = SpectralTarget(x)
        out = multispectral_loss_and_grad(t, r)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    print(f"target + loss/grad (3 resolutions, B=32, T=65536): {s.elapsed_time(e) / 20 * 1000:.1f} us")
else:
    for _ in range(reps):
        t = SpectralTarget(x)
        multispectral_loss_and_grad(t, r)
    torch.cuda.synchronize()
print("ok")
