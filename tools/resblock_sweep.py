"""Time the fused residual-block kernels (GPU dev tool): for each (T, dilation) of the cfg2 model, the fused
forward / backward vs the unfused two-conv path, as HIP-event averages of graph-captured back-to-back launches,
with the HBM bytes each path must move (fused fwd: x + y; fused bwd: dy + x + dx; unfused: per conv in + out
(+ residual / mask operands)).

    python tools/resblock_sweep.py [--batch 32] [--reps 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402


def timed(fn, reps):
    fn()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(5):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / (5 * reps)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--T", type=int, nargs="*", default=[32768, 16384, 8192, 2048])
    p.add_argument("--fused-only", action="store_true", help="skip the unfused two-conv timings")
    a = p.parse_args()
    import vqa_lib as V
    dev = torch.device("cuda", 0)
    C = 32
    for T in a.T:
        for d in (1, 3, 9, 27):
            B = a.batch
            x = torch.randn(B, T, C, device=dev).to(torch.bfloat16)
            dy = torch.randn(B, T, C, device=dev).to(torch.bfloat16)
            wa, wb = torch.randn(3, C, C, device=dev) * 0.1, torch.randn(3, C, C, device=dev) * 0.1
            ba, bb = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
            y, dx, h, dh = (torch.empty_like(x) for _ in range(4))
            gw = [torch.empty(3, C, C, device=dev), torch.empty(C, device=dev)] * 2
            unit = x.numel() * 2
            f_us = timed(lambda: V.resblock_fwd(x, wa, ba, wb, bb, y, d), a.reps)
            dfr = V.Deferred()
            b_us = timed(lambda: V.resblock_bwd(dy, x, wa, ba, wb, bb, dx, *gw, d, dfr), a.reps)
            dfr.descs, dfr.keep = [], []

            def unf_f():
                V.conv1d_fwd(x, wa, ba, None, h, B, T, T, C, C, 3, 1, d, d, V.PRE_RELU, V.BF16)
                V.conv1d_fwd(h, wb, bb, x, y, B, T, T, C, C, 3, 1, 1, 1, V.PRE_RELU | V.ADD_RESIDUAL, V.BF16)

            def unf_b():
                V.conv1d_bwd_data_weight(dy, wb, h, None, dh, gw[2], gw[3], B, T, T, C, C, 3, 1, 1, 1, V.PRE_RELU,
                                         V.BF16, dfr)
                V.conv1d_bwd_data_weight(dh, wa, x, dy, dx, gw[0], gw[1], B, T, T, C, C, 3, 1, d, d,
                                         V.PRE_RELU | V.ADD_RESIDUAL, V.BF16, dfr)
            if a.fused_only:
                print(f"T={T:6d} d={d:2d}  fused fwd {f_us:7.1f} us ({2 * unit / f_us / 1e3:5.0f} GB/s)  "
                      f"bwd {b_us:7.1f} us ({3 * unit / b_us / 1e3:5.0f} GB/s)", flush=True)
                continue
            uf_us = timed(unf_f, a.reps)
            ub_us = timed(unf_b, a.reps)
            dfr.descs, dfr.keep = [], []
            print(f"T={T:6d} d={d:2d}  fused fwd {f_us:7.1f} us ({2 * unit / f_us / 1e3:5.0f} GB/s)  "
                  f"bwd {b_us:7.1f} us ({3 * unit / b_us / 1e3:5.0f} GB/s) | unfused fwd {uf_us:7.1f} us "
                  f"({5 * unit / uf_us / 1e3:5.0f} GB/s) bwd {ub_us:7.1f} us ({7 * unit / ub_us / 1e3:5.0f} GB/s)",
                  flush=True)


if __name__ == "__main__":
    main()
