"""Phase timing of the fused residual-block backward from in-kernel s_memtime stamps (GPU dev tool).

Needs a library built with -DVQA_RS_STAMPS (tools/mkvar.sh stamps "-DVQA_RS_STAMPS" vqa_resblock.hip), passed as
VQA_LIB_PATH. Every wave stamps 8 points of its workgroup's 5th tile; this prints, per team (W = waves 0-1, H = 2-3),
the median cycles of: h recompute | barrier | phase 2 (dW_b / dh) | barrier | staging wait | phase 3 (dx / dW_a) |
tail (barrier, staging store, next loads, barrier) and the whole tile.

    VQA_LIB_PATH=variants/stamps.so python tools/rs_stamps.py [--T 32768] [--d 9 27] [--batch 32]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

NAMES = ["h", "bar1", "ph2", "bar2", "wait", "ph3", "tail"]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--T", type=int, default=32768)
    p.add_argument("--d", type=int, nargs="*", default=[9, 27])
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--fwd", action="store_true", help="stamp the forward: start | conv_a + H | barrier | staging | "
                   "conv_b + y | barrier")
    a = p.parse_args()
    import vqa_lib as V
    L = V.lib()
    L.vqa_rs_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    dev = torch.device("cuda", 0)
    C, B, T = 32, a.batch, a.T
    x = torch.randn(B, T, C, device=dev).to(torch.bfloat16)
    dy = torch.randn(B, T, C, device=dev).to(torch.bfloat16)
    wa, wb = torch.randn(3, C, C, device=dev) * 0.1, torch.randn(3, C, C, device=dev) * 0.1
    ba, bb = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    dx = torch.empty_like(x)
    gw = [torch.empty(3, C, C, device=dev), torch.empty(C, device=dev)] * 2
    for d in a.d:
        for _ in range(3):
            if a.fwd:
                V.resblock_fwd(x, wa, ba, wb, bb, dx, d)
            else:
                dfr = V.Deferred()
                V.resblock_bwd(dy, x, wa, ba, wb, bb, dx, *gw, d, dfr)
            torch.cuda.synchronize()
        n = 1024 * 4 * 8
        buf = (ctypes.c_ulonglong * n)()
        assert L.vqa_rs_stamps(buf, n) == n
        s = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(1024, 4, 8)
        last = 5 if a.fwd else 7
        live = (s[:, :, last] > s[:, :, 0]).all(axis=1) & (s[:, :, 0] > 0).all(axis=1)
        s = s[live][:, :, :last + 1]
        dlt = np.diff(s, axis=2)  # [wg][wave][phases]
        tot = s[:, :, last] - s[:, :, 0]
        if a.fwd:
            med = np.median(dlt.reshape(-1, last), axis=0)
            print(f"T={T} d={d} forward: {len(s)} workgroups; " + "  ".join(
                f"{k} {v:6.0f}" for k, v in zip(["conv_a", "bar1", "staging", "conv_b", "bar2"], med)) +
                f" | tile {np.median(tot):6.0f}", flush=True)
            continue
        print(f"T={T} d={d}: {len(s)} workgroups stamped (median cycles per phase)")
        for team, w in (("W", [0, 1]), ("H", [2, 3])):
            med = np.median(dlt[:, w, :].reshape(-1, 7), axis=0)
            print(f"  team {team}: " + "  ".join(f"{k} {v:6.0f}" for k, v in zip(NAMES, med)) +
                  f"  | tile {np.median(tot[:, w]):6.0f}")
        # how far apart the workgroup's waves enter the tile
        skew = s[:, :, 0].max(axis=1) - s[:, :, 0].min(axis=1)
        print(f"  entry skew median {np.median(skew):.0f}, tile p10/p90 {np.percentile(tot, 10):.0f}/"
              f"{np.percentile(tot, 90):.0f}", flush=True)
        V.Deferred().descs = []


if __name__ == "__main__":
    main()
