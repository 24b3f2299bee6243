"""Keras Adam launch on a parameter-sized flat buffer (GPU dev tool): time per launch, and the updated weights /
moments saved or compared bitwise with another build's (--save / --check).

    [VQA_LIB_PATH=...] python tools/adam_check.py [--n 968835] [--save OUT.pt | --check OUT.pt]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=968835)
    ap.add_argument("--save")
    ap.add_argument("--check")
    a = ap.parse_args()
    import vqa_lib as V
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(3)
    w, g = (torch.randn(a.n, device=dev, generator=gen) for _ in range(2))
    m, v = torch.zeros_like(w), torch.zeros_like(w)
    it = torch.zeros(1, dtype=torch.int64, device=dev)
    for _ in range(3):
        V.adam_keras(w, g, m, v, it, 1e-3, 0.9, 0.999, 1e-7, 0.5)
        V.counter_add(it, 1)
    torch.cuda.synchronize()
    out = {"w": w.cpu(), "m": m.cpu(), "v": v.cpu()}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(50):
        V.adam_keras(w, g, m, v, it, 1e-3, 0.9, 0.999, 1e-7, 0.5)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / 50
    print(f"adam n={a.n}: {us:.1f} us per launch ({7 * 4 * a.n / us / 1e3:.0f} GB/s)", flush=True)
    if a.save:
        torch.save(out, a.save)
    if a.check:
        ref = torch.load(a.check, weights_only=True)
        print("bitwise vs saved:", {k: bool(torch.equal(out[k], ref[k])) for k in out}, flush=True)


if __name__ == "__main__":
    main()
