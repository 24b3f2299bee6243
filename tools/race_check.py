"""Stream-race probe (GPU dev tool): the benched architecture (cfg2 form on a short chunk, bf16, level
streams) trained one step from the same state several times, on the default stream and on a side stream;
the exchanged-bucket gradients must be bitwise equal across every run.

    python tools/race_check.py [reps] [batch]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT, os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import dp_worker as W  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
xs = [x[:B] for x in W.batches(2, "cfg2_short")]
ref = None
for mode in ["default", "side"] * reps:
    m = W.build(B, config="cfg2_short", dtype=os.environ.get("DT", "bf16"))
    x = m._as_input(xs[0])
    if mode == "side":
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m._compute(x, True)
        torch.cuda.current_stream().wait_stream(s)
    else:
        m._compute(x, True)
    torch.cuda.synchronize()
    P = m.layout["grads"][1]
    g = m.bucket[:P].detach().cpu().clone()
    if ref is None:
        ref = g
    diff = (g - ref).abs()
    nbad = int((diff > 0).sum())
    print(f"{mode:8s} max|dg| {float(diff.max()):.3e}  elements differing {nbad} of {g.numel()}", flush=True)
    if nbad:
        idx = torch.nonzero(diff > 0).flatten()
        print("   first differing indices:", idx[:8].tolist(), "last:", idx[-4:].tolist())
    del m
    torch.cuda.empty_cache()
