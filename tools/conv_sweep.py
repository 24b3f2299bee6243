"""Per-call timing of every libvqa conv launch in one eager cfg2 train step (GPU dev tool).

Wraps vqa_lib's conv entry points with HIP events on the launch stream, groups calls by shape, and
prints time and algorithmic GB/s (inputs + outputs + epilogue operands, activation dtype) per group,
plus a device-to-device copy of 128 MB as the achievable-bandwidth yardstick.

    python tools/conv_sweep.py [--batch 32] [--seq 65536] [--reps 3]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--seq", type=int, default=65536)
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    import vqa_lib as V
    from bench import CFG2
    from data_utils import synthetic_batch
    from vqvae import VQVAE

    dev = torch.device("cuda", 0)
    m = VQVAE((a.seq, 1), dtype="bf16", device=dev, **CFG2)
    m.compile()
    x = torch.from_numpy(synthetic_batch(a.batch, a.seq, seed=1)).to(dev)
    m.train_step(x)
    torch.cuda.synchronize()

    calls = collections.OrderedDict()  # shape key -> (entry point, args, calls per step)
    names = ["conv1d_fwd", "conv1d_bwd_data", "conv1d_transpose_fwd", "conv1d_transpose_bwd_data",
             "conv1d_bwd_weight_deferred", "conv1d_transpose_bwd_weight_deferred", "conv1d_bwd_data_weight"]
    orig = {n: getattr(V, n) for n in names}

    def wrap(n):
        f = orig[n]

        def g(*args):
            ts = [t for t in args if isinstance(t, torch.Tensor)]
            ints = [v for v in args if isinstance(v, int)]
            key = (n,) + tuple(ints[:10])
            if key in calls:
                calls[key][2] += 1
            else:
                calls[key] = [n, args, 1]
            return f(*args)
        return g

    for n in names:
        setattr(V, n, wrap(n))
    m._compute(x, True)
    torch.cuda.synchronize()
    for n in names:
        setattr(V, n, orig[n])

    # time each distinct call as 10 back-to-back launches inside a hipGraph (no host gaps)
    res = []
    for key, (n, args, cnt) in calls.items():
        nbytes = sum(t.numel() * t.element_size() for t in args if isinstance(t, torch.Tensor) and t.numel() > 4096)

        def run():
            if n.endswith("_deferred") or n == "conv1d_bwd_data_weight":
                orig[n](*args[:-1], V.Deferred())
            else:
                orig[n](*args)
        run()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(10):
                run()
        g.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            g.replay()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / (10 * a.reps)
        res.append((us * cnt / 1e3, cnt, us, nbytes, key))
    tot = sum(r[0] for r in res)
    print(f"conv total {tot:.3f} ms/step ({sum(r[1] for r in res)} calls)")
    for ms, cnt, us, nb, key in sorted(res, key=lambda r: -r[0])[:45]:
        print(f"{ms:7.3f} ms/step {cnt:3d}x {us:8.1f} us {nb / 1e6:7.1f} MB {nb / us / 1e3:7.0f} GB/s  {key}")

    src = torch.empty(64 * 1024 * 1024, dtype=torch.bfloat16, device=dev)
    dst = torch.empty_like(src)
    for _ in range(3):
        dst.copy_(src)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        dst.copy_(src)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / 20
    print(f"d2d copy 128 MB read + 128 MB write: {us:.1f} us = {2 * src.numel() * 2 / us / 1e3:.0f} GB/s")


if __name__ == "__main__":
    main()
