"""Is the config-2 step bound by a critical path or by total kernel work? (GPU dev tool)

A spin of S cycles (torch.cuda._sleep: one workgroup, no memory traffic) is queued in front of every launch of the
named libvqa entry points while the step is captured; the spins then sit on those launches' streams in every
replay. If the step is critical-path-bound through them it grows by about the spin time per delayed launch on
the path; if it is bound by total kernel work it barely moves (a spin occupies one CU slot).

    python tools/critpath.py [--cycles 200000] [--steps 20] ENTRY [ENTRY ...]   (e.g. vq_ema_apply_derived)
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("entries", nargs="*")
    p.add_argument("--cycles", type=int, default=200_000)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--levels", type=str, default="", help="only launches on these levels' streams (e.g. 1,2)")
    p.add_argument("--first", action="store_true", help="only the first matching launch per level and capture")
    a = p.parse_args()
    import vqa_lib
    from bench import CFG2
    from data_utils import synthetic_batch_device
    from vqvae import VQVAE

    dev = torch.device("cuda", 0)
    # the spin's own length at the shader clock
    torch.cuda._sleep(a.cycles)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        torch.cuda._sleep(a.cycles)
    torch.cuda.synchronize()
    spin_us = (time.perf_counter() - t) / 10 * 1e6
    x = [synthetic_batch_device(32, 65536, seed=1234 + 7919 * i, rank=0, device=dev) for i in range(2)]

    def run(entries):
        m = VQVAE((65536, 1), dtype="bf16", device=dev, **CFG2)
        m.compile()
        hits = [0]
        lv = [int(v) for v in a.levels.split(",") if v != ""]
        seen = set()

        def hook():
            if sys._getframe(2).f_code.co_name not in entries:  # the vqa_lib entry that called stream()
                return
            if not torch.cuda.is_current_stream_capturing():  # only the replayed graph carries spins
                return
            cur = torch.cuda.current_stream()
            streams = m._streams or []
            level = next((i for i, st in enumerate(streams) if st.cuda_stream == cur.cuda_stream), None)
            if lv and level not in lv:
                return
            if a.first:
                if level in seen:
                    return
                seen.add(level)
            hits[0] += 1
            torch.cuda._sleep(a.cycles)

        vqa_lib.launch_hook = hook if entries else None
        try:
            m.capture_train_step(x[0], warmup=1)
        finally:
            vqa_lib.launch_hook = None
        for i in range(3):
            m.train_step(x[i % 2])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            m.train_step(x[i % 2])
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        del m
        torch.cuda.empty_cache()
        return ms, hits[0]

    base, _ = run([])
    hit_ms, hits = run(set(a.entries))
    base2, _ = run([])
    print(f"spin {spin_us:.1f} us; delayed entries {sorted(a.entries)} levels {a.levels or 'all'}"
          f"{' first only' if a.first else ''}: {hits} spins in the graph")
    print(f"step: {base:.3f} / {base2:.3f} ms without, {hit_ms:.3f} ms with -> +{hit_ms - (base + base2) / 2:.3f} ms",
          flush=True)


if __name__ == "__main__":
    main()
