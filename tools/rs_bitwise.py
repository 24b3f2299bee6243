"""Residual-block kernels of two library builds, output for output (GPU dev tool).

    python tools/rs_bitwise.py --save FILE      (the library in VQA_LIB_PATH, or the in-tree one)
    python tools/rs_bitwise.py --check FILE     (another build: every output must be bitwise the saved one)

Shapes: every dilation of the model at the config-2 lengths (B = 32 at T = 32768 / 8192 / 2048 / 512 for the
backward's two tile plans), ragged and short items, bf16 and fp32; seeded inputs as tests/test_gpu_resblock.py draws
them (x, dy ~ N(0, 1), glorot-scaled weights, small biases). Outputs: forward y, backward dx, dW_a, db_a, dW_b, db_b.
Large outputs are kept as sha256 digests, small ones whole (so a mismatch can be counted and located).
"""
import argparse
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402

import vqa_lib as V  # noqa: E402

C = 32
SHAPES = [(32, 32768, d) for d in (1, 3, 9, 27)] + [(32, 8192, 9), (32, 4096, 3), (32, 2048, 27), (32, 512, 1),
                                                   (3, 1000, 9), (2, 4097, 27), (1, 100, 27), (5, 2500, 3)]
SMALL = 1 << 21  # outputs up to 2 MB are kept whole


def block(B, T, d, seed, dt, dev):
    g = torch.Generator(device=dev).manual_seed(seed)
    r = lambda *s: torch.randn(*s, generator=g, device=dev)  # noqa: E731
    p = dict(x=r(B, T, C).to(dt), dy=r(B, T, C).to(dt), wa=r(3, C, C) / (3 * C) ** 0.5, wb=r(3, C, C) / (3 * C) ** 0.5,
             ba=0.1 * r(C), bb=0.1 * r(C))
    return p


def run(shapes, dts):
    dev = torch.device("cuda", 0)
    out = {}
    for dt in dts:
        for i, (B, T, d) in enumerate(shapes):
            if dt == torch.float32 and B * T > 32 * 8192:
                continue
            p = block(B, T, d, 100 + i, dt, dev)
            y = torch.empty_like(p["x"])
            V.resblock_fwd(p["x"], p["wa"], p["ba"], p["wb"], p["bb"], y, d)
            dx = torch.empty_like(p["x"])
            g = [torch.empty(3, C, C, device=dev), torch.empty(C, device=dev), torch.empty(3, C, C, device=dev),
                 torch.empty(C, device=dev)]
            V.resblock_bwd(p["dy"], p["x"], p["wa"], p["ba"], p["wb"], p["bb"], dx, *g, d)
            torch.cuda.synchronize()
            for name, t in (("y", y), ("dx", dx), ("dwa", g[0]), ("dba", g[1]), ("dwb", g[2]), ("dbb", g[3])):
                key = f"{str(dt)[6:]} B{B} T{T} d{d} {name}"
                c = t.detach().cpu().contiguous()
                raw = c.view(torch.uint8) if c.dtype != torch.bfloat16 else c.view(torch.int16).view(torch.uint8)
                out[key] = (hashlib.sha256(raw.numpy().tobytes()).hexdigest(), c if raw.numel() <= SMALL else None)
            del p, y, dx, g
            torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--save")
    ap.add_argument("--check")
    a = ap.parse_args()
    res = run(SHAPES, [torch.bfloat16, torch.float32])
    if a.save:
        torch.save(res, a.save)
        print(f"saved {len(res)} outputs from {V.LIB_PATH}")
        return 0
    ref = torch.load(a.check, weights_only=True)
    bad = 0
    for k, (h, t) in ref.items():
        h2, t2 = res[k]
        if h == h2:
            continue
        bad += 1
        if t is not None and t2 is not None:
            n = int((t.view(torch.int16 if t.dtype == torch.bfloat16 else torch.int32) !=
                     t2.view(torch.int16 if t2.dtype == torch.bfloat16 else torch.int32)).sum())
            m = float((t.double() - t2.double()).abs().max())
            print(f"DIFF {k}: {n} of {t.numel()} elements, max |diff| {m:.3e}")
        else:
            print(f"DIFF {k} (digest)")
    print(f"{V.LIB_PATH}: {len(ref) - bad} of {len(ref)} outputs bitwise equal")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
