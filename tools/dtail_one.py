"""Decoder-tail launch times at the config-2 shape (GPU dev tool): python tools/dtail_one.py [--reps N].

B = 32 items of T = 32768 rows (the waveform end of every level's decoder: h [B, T, 32] bf16 -> y [B, 2T]), the
forward and the backward (its launch sequence: compose, the row kernel, the partial reductions, the chain) timed
with events around N back-to-back calls each, after a warm-up; the library is VQA_LIB_PATH's (or the in-tree one).
Also prints a digest of the backward's outputs, so two builds can be compared for bitwise equality.
"""
import argparse
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402

import vqa_lib as V  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--T", type=int, default=32768)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    h = torch.randn(a.B, a.T, 32, generator=g, device=dev).to(torch.bfloat16)
    dy = torch.randn(a.B, 2 * a.T, 1, generator=g, device=dev)
    p = [torch.randn(4, 64, 32, generator=g, device=dev) * 0.1, torch.randn(64, generator=g, device=dev) * 0.1,
         torch.randn(3, 64, 1, generator=g, device=dev) * 0.1, torch.randn(1, generator=g, device=dev) * 0.1]
    y = torch.empty(a.B, 2 * a.T, 1, device=dev)
    dh = torch.empty_like(h)
    grads = [torch.empty_like(t) for t in p]
    fwd = lambda: V.dtail_fwd(h, *p, y)  # noqa: E731
    bwd = lambda: V.dtail_bwd(dy, h, *p, dh, *grads)  # noqa: E731
    for f, name in ((fwd, "fwd"), (bwd, "bwd")):
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        byt = a.B * a.T * 32 * 2 + a.B * 2 * a.T * 4 + (a.B * a.T * 32 * 2 if name == "bwd" else 0)
        print(f"dtail_{name} B={a.B} T={a.T}: {us:7.2f} us per call ({byt / us / 1e6:.2f} TB/s algorithmic)")
    torch.cuda.synchronize()
    dig = hashlib.sha256()
    for t in [y, dh] + grads:
        c = t.detach().cpu().contiguous()
        dig.update((c.view(torch.int16) if c.dtype == torch.bfloat16 else c.view(torch.int32)).numpy().tobytes())
    print(f"digest {dig.hexdigest()[:16]} ({V.LIB_PATH})")


if __name__ == "__main__":
    main()
