"""Is the spectral loss gradient chain repeatable while another process shares the GPU? (GPU dev tool)

Each worker computes the target spectrograms of one batch once, then runs vqa_spectral_loss_target on the same
(target, reconstruction) REPS times and compares every repeat with the first: the gradient dr, and the loss
workspace region by region (per resolution: frame gradients `fg`, per-frame partials `part`; then the per-item
losses / scales). `python tools/spec_race.py NPROC REPS` runs NPROC workers at once (1 = alone).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402


def a64(n):
    return (n + 63) // 64 * 64


def worker(reps, wid):
    import vqa_lib as V
    from data_utils import STFT_ARGS
    dev = torch.device("cuda", 0)
    B, T = 32, 65536
    g = torch.Generator(device="cpu").manual_seed(3)
    x = (torch.randn(B, T, generator=g) * 0.3).to(dev)
    r = (0.5 * x.cpu() + 0.2 * torch.randn(B, T, generator=g)).to(dev)
    tg = V.spectral_target(x, *STFT_ARGS)
    n_fft, hop, win = STFT_ARGS
    ws = V.workspace(V.spectral_loss_target_workspace(B, T, n_fft, hop, win, True), dev)
    regions, o = [], 0
    for i in range(len(n_fft)):
        F = 1 + (T - win[i]) // hop[i]
        regions.append((f"fg{n_fft[i]}", o, B * F * win[i]))
        o += a64(B * F * win[i])
        regions.append((f"part{n_fft[i]}", o, B * F * 2))
        o += a64(B * F * 2)
    regions.append(("tail", o, B * len(n_fft) * 2))
    first = None
    bad = {}
    for k in range(reps):
        loss = torch.empty(1, device=dev)
        dr = torch.empty(B, T, device=dev)
        ws.zero_()
        V.spectral_loss_target(tg, r, loss, dr, None, n_fft, hop, win, ws=ws)
        torch.cuda.synchronize()
        wf = ws.view(torch.float32)
        snap = {"dr": dr.cpu(), "loss": loss.cpu()}
        for name, off, n in regions:
            snap[name] = wf[off:off + n].cpu()
        if first is None:
            first = snap
            continue
        for key, v in snap.items():
            d = int((v != first[key]).sum())
            if d:
                bad.setdefault(key, []).append(d)
    print(f"worker {wid}: {reps - 1} repeats vs the first; differing elements per region: "
          f"{ {k: (len(v), max(v)) for k, v in bad.items()} or 'none'}", flush=True)


def main():
    nproc, reps = int(sys.argv[1]), int(sys.argv[2])
    if nproc == 1:
        worker(reps, 0)
        return
    procs = [subprocess.Popen([sys.executable, __file__, "--worker", str(reps), str(i)]) for i in range(nproc)]
    rc = [p.wait(timeout=600) for p in procs]
    if any(rc):
        sys.exit(1)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--worker":
        worker(int(sys.argv[2]), int(sys.argv[3]))
    else:
        main()
