"""When does each level's chain end inside the config-2 step? (GPU dev tool; orders VQA_DP_OVERLAP_ORDER)

Eager step with the levels on their streams; an event at the fork and one at the end of each level's chain (before
the join) give each chain's length; the levels' exchanges are best issued in the order their chains end.
    python tools/level_ends.py [--steps 5]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=5)
    a = p.parse_args()
    from bench import CFG2
    from data_utils import synthetic_batch_device
    import vqvae as VV
    dev = torch.device("cuda", 0)
    m = VV.VQVAE((65536, 1), dtype="bf16", device=dev, **CFG2)
    m.compile()
    x = synthetic_batch_device(32, 65536, seed=1234, rank=0, device=dev)
    ends = {}
    orig = m._level_step

    def timed(x_, l, *args, **kw):
        orig(x_, l, *args, **kw)
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ends[l] = e
    m._level_step = timed
    for it in range(a.steps + 2):
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t0.record()
        m.train_step(x)
        t1 = torch.cuda.Event(enable_timing=True)
        t1.record()
        torch.cuda.synchronize()
        if it >= 2:
            print("step %.3f ms; chain ends " % t0.elapsed_time(t1) +
                  "  ".join(f"level {l} {t0.elapsed_time(ends[l]):.3f}" for l in sorted(ends)), flush=True)


if __name__ == "__main__":
    main()
