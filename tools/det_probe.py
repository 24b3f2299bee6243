"""Is one process's local gradient bitwise reproducible — in the same process (a second model), and in a fresh
process, and after other model shapes ran first? (GPU dev tool for the DP exchange tests.)

    python tools/det_probe.py CONFIG DTYPE B [--child OUT]
Prints, for each comparison, the number of differing gradient elements and the worst parameters.
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT, os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import dp_worker as W  # noqa: E402


def local_grad(config, dtype, B, side_stream=False):
    W.B_LOCAL = B
    m = W.build(B, config=config, dtype=dtype)
    x = W.batches(2, config)[0][:B]
    if side_stream:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m._compute(m._as_input(x), True)
        torch.cuda.current_stream().wait_stream(s)
    else:
        m._compute(m._as_input(x), True)
    torch.cuda.synchronize()
    g = m.bucket[:m.layout["grads"][1]].detach().cpu().clone()
    offs = {k: (int(o), int(torch.Size(sh).numel())) for k, (o, sh) in m.store.offsets.items()}
    del m
    torch.cuda.empty_cache()
    return g, offs


def report(name, a, b, offs):
    n = int((a != b).sum())
    line = f"{name:28s} {n:8d} of {a.numel()} differ"
    if n:
        gmax = float(b.double().abs().max())
        per = sorted(((float((a[o:o + k].double() - b[o:o + k].double()).abs().max()) / gmax, int((a[o:o + k] != b[o:o + k]).sum()), nm)
                      for nm, (o, k) in offs.items()), reverse=True)[:5]
        line += "  worst: " + ", ".join(f"{nm} {v:.1e} ({c})" for v, c, nm in per)
    print(line, flush=True)


def main():
    config, dtype, B = sys.argv[1], sys.argv[2], int(sys.argv[3])
    if len(sys.argv) > 5 and sys.argv[4] == "--child":
        g, _ = local_grad(config, dtype, B)
        torch.save(g, sys.argv[5])
        return
    g0, offs = local_grad(config, dtype, B)
    g1, _ = local_grad(config, dtype, B)
    report("same process, 2nd model", g1, g0, offs)
    g2, _ = local_grad(config, dtype, B, side_stream=True)
    report("same process, side stream", g2, g0, offs)
    out = os.path.join(tempfile.gettempdir(), "det_probe_child.pt")
    subprocess.run([sys.executable, __file__, config, dtype, str(B), "--child", out], check=True)
    report("fresh process", torch.load(out, weights_only=True), g0, offs)
    local_grad(config, dtype, 2 * B)  # another batch shape first
    g3, _ = local_grad(config, dtype, B)
    report("after a 2B model", g3, g0, offs)


if __name__ == "__main__":
    main()
