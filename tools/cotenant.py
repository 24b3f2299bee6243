"""Wrong results when a second process shares the GPU: product race or platform? (GPU dev tool, round 5)

Round 4 recorded a single process's step gradient that is bitwise repeatable alone and differs beside a second
process, only while the product's level streams overlap. Two explanations fit that record: a
missing cross-stream dependency in the product whose window only opens under the neighbour's timing, or the
platform corrupting waves of a process whose several hardware queues are active while another process runs.
This tool separates them:

    inject  CONFIG DTYPE B N [P]   product ALONE: one reference step with the levels serialised (one stream),
                                   then N steps with the level streams overlapping and, before every libvqa
                                   launch with probability P, a random 10-400 us spin on the launching stream
                                   (vqa_lib.launch_hook) — every cross-stream order the step relies on is
                                   stretched both ways. A missing dependency shows as a differing gradient.
    product CONFIG DTYPE B N [--hog K] [--serial]
                                   the product's local gradient N times vs the first, beside a hog process with
                                   K concurrent streams (0 = alone); --serial runs the levels on one stream.
    control N [--hog K]            no product code: a deterministic torch workload on 3 concurrent streams (fp32
                                   GEMMs, row reductions, elementwise chains) N times vs the first, beside the hog.
    kernel N [--hog K] [--streams S]
                                   single libvqa kernels (decoder tail, residual-block forward, spectral loss +
                                   gradient; config-2 level-0 sizes) on S streams, N iterations on the same
                                   inputs, beside the hog: every output vs the first.
    hog K SECONDS                  the neighbour: bf16 8192^2 matmuls on K concurrent streams.
"""
import os
import random
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT, os.path.join(ROOT, "tests")]

import torch  # noqa: E402


def hog(k, seconds):
    streams = [torch.cuda.Stream() for _ in range(k)]
    mats = [torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16) for _ in range(k)]
    t0 = time.time()
    while time.time() - t0 < seconds:
        for s, i in zip(streams, range(k)):
            with torch.cuda.stream(s):
                for _ in range(10):
                    mats[i] = (mats[i] @ mats[i]).clamp_(-1, 1)
        torch.cuda.synchronize()


def start_hog(k):
    if k <= 0:
        return None
    p = subprocess.Popen([sys.executable, __file__, "hog", str(k), "300"])
    time.sleep(8)  # the neighbour's torch import and first launches
    return p


def local_grad(config, dtype, B, serial=False, hook=None):
    import dp_worker as W
    import vqa_lib
    W.B_LOCAL = B
    m = W.build(B, config=config, dtype=dtype)
    m.concurrent_levels = not serial
    x = m._as_input(W.batches(1, config)[0][:B])
    torch.cuda.synchronize()
    vqa_lib.launch_hook = hook
    try:
        m._compute(x, True)
    finally:
        vqa_lib.launch_hook = None
    torch.cuda.synchronize()
    g = m.bucket.detach().cpu().clone()  # grads | EMA sums, reset rows | losses
    P = m.layout["grads"][1]
    offs = {k: (int(o), int(torch.Size(sh).numel())) for k, (o, sh) in m.store.offsets.items()}
    del m
    torch.cuda.empty_cache()
    return g, P, offs


def report(name, a, b, P, offs):
    n, ns = int((a[:P] != b[:P]).sum()), int((a[P:] != b[P:]).sum())
    line = f"{name:40s} grads {n:8d} of {P} differ, stats/losses {ns:6d} of {a.numel() - P}"
    if n:
        gmax = float(b[:P].double().abs().max())
        per = sorted(((float((a[o:o + k].double() - b[o:o + k].double()).abs().max()) / gmax,
                       int((a[o:o + k] != b[o:o + k]).sum()), nm) for nm, (o, k) in offs.items()), reverse=True)[:4]
        line += "  worst: " + ", ".join(f"{nm} {v:.1e} ({c})" for v, c, nm in per)
    print(line, flush=True)
    return n + ns


def delay_hook(rng, p):
    def hook():
        if rng.random() < p:
            torch.cuda._sleep(rng.randint(25_000, 1_000_000))  # ~10-400 us at the shader clock
    return hook


def cmd_inject(config, dtype, B, n, p=0.15):
    ref, P, offs = local_grad(config, dtype, B, serial=True)
    bad = 0
    for i in range(n):
        g, _, _ = local_grad(config, dtype, B, hook=delay_hook(random.Random(1000 + i), p))
        bad += report(f"concurrent levels + delays, pattern {i}", g, ref, P, offs) > 0
    g, _, _ = local_grad(config, dtype, B)
    bad += report("concurrent levels, no delays", g, ref, P, offs) > 0
    print(f"SUMMARY inject {config} {dtype} B={B}: {bad} of {n + 1} concurrent runs differ from the serial step")
    return bad


def cmd_product(config, dtype, B, n, k, serial):
    bg = start_hog(k)
    try:
        g0, P, offs = local_grad(config, dtype, B, serial=serial)
        bad = 0
        for i in range(1, n):
            g, _, _ = local_grad(config, dtype, B, serial=serial)
            bad += report(f"rep {i} ({'serial' if serial else 'concurrent'} levels, hog {k})", g, g0, P, offs) > 0
    finally:
        if bg is not None:
            bg.kill()
            bg.wait()
    print(f"SUMMARY product {config} {dtype} B={B} serial={serial} hog={k}: {bad} of {n - 1} repeats differ")
    return bad


def control_once():
    torch.manual_seed(0)
    streams = [torch.cuda.Stream() for _ in range(3)]
    xs = [torch.randn(4096, 1024, device="cuda") for _ in range(3)]
    ws = [torch.randn(1024, 1024, device="cuda") / 32 for _ in range(3)]
    torch.cuda.synchronize()
    outs = [[] for _ in range(3)]
    for s, i in zip(streams, range(3)):
        with torch.cuda.stream(s):
            x = xs[i]
            for _ in range(60):
                x = torch.tanh(x @ ws[i]) * 1.5 + 0.01
                x = x - x.mean(dim=-1, keepdim=True)
                outs[i].append(x.pow(2).sum(dim=-1))
    torch.cuda.synchronize()
    return torch.cat([torch.cat(o) for o in outs]).cpu()


def cmd_control(n, k):
    bg = start_hog(k)
    try:
        r0 = control_once()
        bad = 0
        for i in range(1, n):
            r = control_once()
            d = int((r != r0).sum())
            print(f"control rep {i} (hog {k}): {d} of {r.numel()} differ", flush=True)
            bad += d > 0
    finally:
        if bg is not None:
            bg.kill()
            bg.wait()
    print(f"SUMMARY control hog={k}: {bad} of {n - 1} repeats differ")
    return bad


def cmd_kernel(n, k, streams, ops=("dtail", "resblock", "spectral")):
    """Single libvqa kernels (the decoder tail, the residual-block forward and the spectral loss + gradient at the
    config-2 level-0 sizes) on `streams` concurrent streams, n iterations each on the SAME inputs, beside the hog:
    every output vs the first."""
    import vqa_lib as V
    from data_utils import STFT_ARGS, SpectralTarget
    g = torch.Generator(device="cuda").manual_seed(5)
    B, T, C = 32, 32768, 32
    h = (torch.randn(B, T, C, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    w_up = torch.randn(4, 64, C, device="cuda", generator=g) * 0.1
    b_up = torch.randn(64, device="cuda", generator=g) * 0.1
    w_out = torch.randn(3, 64, 1, device="cuda", generator=g) * 0.1
    b_out = torch.randn(1, device="cuda", generator=g) * 0.1
    wa, wb = (torch.randn(3, C, C, device="cuda", generator=g) * 0.1 for _ in range(2))
    ba, bb = (torch.randn(C, device="cuda", generator=g) * 0.1 for _ in range(2))
    import data_utils as DU
    x = DU.synthetic_batch_device(B, 2 * T)
    tgt = SpectralTarget(x)
    r = (x.view(B, 2 * T) + 0.01 * torch.randn(B, 2 * T, device="cuda", generator=g)).contiguous()
    torch.cuda.synchronize()
    bg = start_hog(k)
    outs = {}
    try:
        ss = [torch.cuda.Stream() for _ in range(streams)]
        for it in range(n):
            for si, s in enumerate(ss):
                with torch.cuda.stream(s):
                    y = torch.zeros(B, 2 * T, 1, device="cuda")
                    if "dtail" in ops:
                        V.dtail_fwd(h, w_up, b_up, w_out, b_out, y)
                    yr = torch.zeros_like(h)
                    if "resblock" in ops:
                        V.resblock_fwd(h, wa, ba, wb, bb, yr, 9)
                    loss = torch.zeros(1, device="cuda")
                    dr = torch.zeros_like(r)
                    if "spectral" in ops:
                        V.spectral_loss_target(tgt.mags, r, loss, dr, None, *STFT_ARGS)
                    outs[(it, si)] = (y, yr, loss, dr)
        torch.cuda.synchronize()
    finally:
        if bg is not None:
            bg.kill()
            bg.wait()
    ref = outs[(0, 0)]
    bad = 0
    for key, o in outs.items():
        diffs = [int((a != b).sum()) for a, b in zip(o, ref)]
        if any(diffs):
            bad += 1
            print(f"iteration {key[0]} stream {key[1]}: differing elements dtail {diffs[0]} resblock {diffs[1]} "
                  f"loss {diffs[2]} spectral grad {diffs[3]}", flush=True)
            if diffs[3]:
                bad_dr = (o[3] != ref[3]).nonzero()
                items = sorted(set(bad_dr[:, 0].tolist()))
                print(f"   spectral grad: items {items}, t {int(bad_dr[:, 1].min())}..{int(bad_dr[:, 1].max())}; first "
                      f"got / want: {[(round(float(o[3][i, t]), 7), round(float(ref[3][i, t]), 7)) for i, t in bad_dr[:4].tolist()]}",
                      flush=True)
            if diffs[0]:
                w = (o[0] != ref[0]).view(B, 2 * T).nonzero()[:8].tolist()
                print("   dtail (item, t) got / want:", [(i, t, round(float(o[0][i, t, 0]), 5),
                                                          round(float(ref[0][i, t, 0]), 5)) for i, t in w], flush=True)
    print(f"SUMMARY kernel streams={streams} hog={k}: {bad} of {len(outs) - 1} launches sets differ")
    return bad


def main():
    a = sys.argv[1:]
    hogk = int(a[a.index("--hog") + 1]) if "--hog" in a else 0
    if a[0] == "hog":
        hog(int(a[1]), float(a[2]))
    elif a[0] == "inject":
        cmd_inject(a[1], a[2], int(a[3]), int(a[4]), float(a[5]) if len(a) > 5 else 0.15)
    elif a[0] == "product":
        cmd_product(a[1], a[2], int(a[3]), int(a[4]), hogk, "--serial" in a)
    elif a[0] == "control":
        cmd_control(int(a[1]), hogk)
    elif a[0] == "kernel":
        cmd_kernel(int(a[1]), hogk, int(a[a.index("--streams") + 1]) if "--streams" in a else 3,
                   a[a.index("--ops") + 1].split(",") if "--ops" in a else ("dtail", "resblock", "spectral"))
    else:
        raise SystemExit(__doc__)


if __name__ == "__main__":
    main()
