"""Time the encoder's first conv (1 -> 32 channels, k4, stride 2, fp32 waveform in, bf16 out) at the cfg2
shape in isolation (GPU dev tool): forward and weight gradient, HIP-event averages of graph-replayed
back-to-back launches, with the bytes each must move.

    python tools/first_conv.py [--batch 32] [--T 65536] [--reps 20]
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
    p.add_argument("--T", type=int, default=65536)
    p.add_argument("--reps", type=int, default=20)
    a = p.parse_args()
    import vqa_lib as V
    dev = torch.device("cuda", 0)
    B, T, O, K, S = a.batch, a.T, 32, 4, 2
    To = T // S
    pad = max((To - 1) * S + K - T, 0) // 2
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(B, T, 1, device=dev, generator=g)
    w = torch.randn(K, 1, O, device=dev, generator=g) * 0.3
    b = torch.randn(O, device=dev, generator=g) * 0.1
    y = torch.empty(B, To, O, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(B, To, O, device=dev, generator=g).to(torch.bfloat16)
    dw, db = torch.empty(K, 1, O, device=dev), torch.empty(O, device=dev)
    fl = V.X_F32
    f_us = timed(lambda: V.conv1d_fwd(x, w, b, None, y, B, T, To, 1, O, K, S, 1, pad, fl, V.BF16), a.reps)
    dfr = V.Deferred()

    def wg():
        V.conv1d_bwd_weight_deferred(x, dy, dw, db, B, T, To, 1, O, K, S, 1, pad, fl, V.BF16, dfr)
        dfr.flush()
    w_us = timed(wg, a.reps)
    mb_f = (x.numel() * 4 + y.numel() * 2) / 1e6
    mb_w = (x.numel() * 4 + dy.numel() * 2) / 1e6
    print(f"first conv B={B} T={T}: fwd {f_us:.1f} us ({mb_f / f_us:.2f} TB/s of {mb_f:.0f} MB)  "
          f"wgrad+reduce {w_us:.1f} us ({mb_w / w_us:.2f} TB/s of {mb_w:.0f} MB)", flush=True)
    import hashlib
    dig = hashlib.sha256()
    for t in (y, dw, db):
        c = t.detach().cpu().contiguous()
        dig.update((c.view(torch.int16) if c.dtype == torch.bfloat16 else c.view(torch.int32)).numpy().tobytes())
    print(f"digest {dig.hexdigest()[:16]} (y, dW, db; {V.LIB_PATH})")


if __name__ == "__main__":
    main()
