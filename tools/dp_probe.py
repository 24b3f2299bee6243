"""DP race probe (GPU dev tool): each rank's LOCAL gradient (the bucket just before the exchange) of the
2-rank gloo run (tests/dp_worker.py setup: cfg2_short, every rank on cuda:0) must equal, bitwise, one process
computing the same rank's half of the batch eagerly on the default stream. Names the parameters that differ.

    python tools/dp_probe.py [reps] [mode] [dtype]        (mode: graph | eager | sidegraph)
"""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT, os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import dp_worker as W  # noqa: E402

CONFIG = "cfg2_short"


def worker(mode, out, dtype):
    import torch.distributed as dist
    import vqa_dp
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = W.build(W.B_LOCAL, config=CONFIG, dtype=dtype)
    xs = [x[rank * W.B_LOCAL:(rank + 1) * W.B_LOCAL] for x in W.batches(world, CONFIG)]
    P = m.layout["grads"][1]
    saved = []
    orig = vqa_dp.exchange

    def probe(bucket, group=None):
        if bucket.numel() > P:
            saved.append(bucket[:P].detach().clone())  # on the producer stream, no host sync
        return orig(bucket, group)

    vqa_dp.exchange = probe
    res = W.run(m, xs, mode)  # exactly the test's sequence; step1 = after the first step (+ the capture)
    torch.save({"local": saved[0].cpu(), "exchanged": res["step1"]["grads"], "offsets": {k: (int(o), int(torch.Size(sh).numel()))
                                               for k, (o, sh) in m.store.offsets.items()}}, out)
    dist.barrier()
    dist.destroy_process_group()


def reference(dtype):
    refs = []
    for r in range(2):
        m = W.build(W.B_LOCAL, config=CONFIG, dtype=dtype)
        x = m._as_input(W.batches(2, CONFIG)[0][r * W.B_LOCAL:(r + 1) * W.B_LOCAL])
        m._compute(x, True)
        torch.cuda.synchronize()
        refs.append(m.bucket[:m.layout["grads"][1]].detach().cpu().clone())
        del m
    torch.cuda.empty_cache()
    return refs


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    mode = sys.argv[2] if len(sys.argv) > 2 else "graph"
    dtype = sys.argv[3] if len(sys.argv) > 3 else "bf16"
    refs = reference(dtype)
    out_dir = os.path.join(ROOT, "gpurun_out", "dp_probe")
    os.makedirs(out_dir, exist_ok=True)
    nbad_runs = 0
    for rep in range(reps):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        procs, outs = [], []
        for r in range(2):
            out = os.path.join(out_dir, f"rank{r}.pt")
            env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen([sys.executable, __file__, "--worker", mode, out, dtype], env=env))
            outs.append(out)
        for p in procs:
            assert p.wait(timeout=300) == 0
        bad = False
        for r, o in enumerate(outs):
            res = torch.load(o, weights_only=True)
            g, ref = res["local"], refs[r]
            d = (g.double() - ref.double()).abs()
            n = int((d > 0).sum())
            line = f"rep {rep} rank {r}: {n} of {g.numel()} gradient elements differ, max {float(d.max()):.3e}"
            if n:
                bad = True
                gmax = float(ref.abs().max())
                per = sorted(((float(d[o:o + k].max()) / gmax, int((d[o:o + k] > 0).sum()), name)
                              for name, (o, k) in res["offsets"].items()), reverse=True)
                per = [p for p in per if p[0] > 0]
                line += f" ({len(per)} params): " + ", ".join(f"{nm} {v:.1e}/{c}" for v, c, nm in per[:8])
            print(line, flush=True)
        ex = [torch.load(o, weights_only=True)["exchanged"] for o in outs]
        want = refs[0] + refs[1]
        for r in range(2):
            d = (ex[r].double() - want.double()).abs()
            n = int((d > 0).sum())
            line = f"rep {rep} rank {r}: exchanged != local0 + local1 at {n} elements, max {float(d.max()):.3e}"
            if n:
                bad = True
                offs = torch.load(outs[0], weights_only=True)["offsets"]
                per = sorted(((float(d[o:o + k].max()), int((d[o:o + k] > 0).sum()), name)
                              for name, (o, k) in offs.items()), reverse=True)
                per = [p for p in per if p[0] > 0]
                line += f" ({len(per)} params): " + ", ".join(f"{nm} {v:.1e}/{c}" for v, c, nm in per[:8])
            print(line, flush=True)
        nbad_runs += bad
    print(f"{nbad_runs} of {reps} runs with a local gradient that differs from the eager single process")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--worker":
        worker(sys.argv[2], sys.argv[3], sys.argv[4])
    else:
        main()
