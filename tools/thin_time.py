"""Time the waveform-end convs of the cfg2 step (GPU dev tool): the first encoder conv (1 -> 32 channels, k4 s2,
fp32 input) forward and weight gradient at B = 32, T = 65536, graph-captured back-to-back launches.

    [VQA_LIB_PATH=variants/X.so] python tools/thin_time.py [--save OUT.pt | --check OUT.pt]
(--check: the forward output and the reduced weight gradient must equal, bitwise, those saved from another build)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402


def timed(fn, reps=20):
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
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--save")
    ap.add_argument("--check")
    args = ap.parse_args()
    import vqa_lib as V
    dev = torch.device("cuda", 0)
    B, T, O = 32, 65536, 32
    gen = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(B, T, 1, device=dev, generator=gen)
    dy = torch.randn(B, T // 2, O, device=dev, generator=gen).to(torch.bfloat16)
    y = torch.empty_like(dy)
    w = torch.randn(4, 1, O, device=dev, generator=gen) * 0.1
    b = torch.randn(O, device=dev, generator=gen) * 0.1
    dw, db = torch.empty_like(w), torch.empty_like(b)
    dfr = V.Deferred()
    f_us = timed(lambda: V.conv1d_fwd(x, w, b, None, y, B, T, T // 2, 1, O, 4, 2, 1, 1, 8, V.BF16))
    w_us = timed(lambda: V.conv1d_bwd_weight_deferred(x, dy, dw, db, B, T, T // 2, 1, O, 4, 2, 1, 1, 8, V.BF16, dfr))
    dfr.descs, dfr.keep = [], []
    nb = x.numel() * 4 + dy.numel() * 2
    print(f"first conv fwd {f_us:6.1f} us ({nb / f_us / 1e3:5.0f} GB/s)  wgrad partials {w_us:6.1f} us "
          f"({nb / w_us / 1e3:5.0f} GB/s)", flush=True)
    # parity of the reduced weight gradient against a float64 reference on a slice of the batch
    V.conv1d_bwd_weight(x, dy, dw, db, B, T, T // 2, 1, O, 4, 2, 1, 1, 8, V.BF16)
    xp = torch.nn.functional.pad(x[..., 0].double(), (1, 1))
    g = dy.double()
    ref = torch.stack([torch.einsum("nt,nto->o", xp[:, k:k + T - 1:2][:, :T // 2], g) for k in range(4)])
    err = float((dw[:, 0, :].double() - ref).abs().max() / ref.abs().max())
    print(f"wgrad rel err vs fp64 {err:.2e}; db err {float((db.double() - g.sum((0, 1))).abs().max()):.2e}", flush=True)
    V.conv1d_fwd(x, w, b, None, y, B, T, T // 2, 1, O, 4, 2, 1, 1, 8, V.BF16)
    torch.cuda.synchronize()
    out = {"y": y.cpu(), "dw": dw.cpu(), "db": db.cpu()}
    if args.save:
        torch.save(out, args.save)
    if args.check:
        ref = torch.load(args.check, weights_only=True)
        print("bitwise vs saved:", {k: bool(torch.equal(out[k], ref[k])) for k in out}, flush=True)


if __name__ == "__main__":
    main()
