"""DP exchange diagnosis (GPU dev tool): where does a wrong exchanged gradient come from?

Two gloo ranks on cuda:0 run tests/dp_worker.py's sequence (cfg2_short, bf16, graph warm-up on a side stream)
with `vqa_dp.exchange` replaced by an instrumented exchange over one of these paths:
  device       dist.all_reduce on the DEVICE bucket (torch-gloo stages it through pinned host memory on a
               high-priority pool stream behind an event on the current stream, copies the sum back there)
  device_sync  the same after hipStreamSynchronize of the current stream (the round-3 intermediate fix)
  host         the product path (vqa_dp.exchange: blocking copy out, CPU all_reduce, copy back)
  emulate      the product path, preceded by an emulation of gloo's staging copy (event on the current
               stream, high-priority stream waits, non_blocking D2H into pinned memory, stream sync)
At the exchange each rank records, for the step's full bucket:
  before   a device copy queued on the current stream at entry (what the collective must read)
  staged   (emulate) the pinned copy the emulated staging read
  after    a device copy queued on the current stream right after the exchange returns (the consumer's view:
           what `_update` / the second graph reads), no host sync
  final    the bucket after a device synchronize
and the driver checks, per rank:  before == single-process local gradient,  staged == before,
after == before0 + before1 (fp32 a+b is commutative, so bitwise),  final == after.
A wrong `after` with a right `final` = consumer ordering; a wrong `final` equal to `after` = a wrong sum
(the staging read the wrong bytes); `final` != `after` = a write after the exchange.

    python tools/dp_diag.py PATH REPS [MODE]
"""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT, os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import dp_worker as W  # noqa: E402

CONFIG, DTYPE = os.environ.get("VQA_DIAG_CONFIG", "cfg2_short"), os.environ.get("VQA_DIAG_DTYPE", "bf16")


def worker(path, mode, out):
    import torch.distributed as dist
    import vqa_dp
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = W.build(W.B_LOCAL, config=CONFIG, dtype=DTYPE)
    xs = [x[rank * W.B_LOCAL:(rank + 1) * W.B_LOCAL] for x in W.batches(world, CONFIG)]
    P = m.layout["grads"][1]
    rec = []
    orig = vqa_dp.exchange

    def diag(bucket, group=None):
        if bucket.numel() <= P or rec:  # instrument the first full-bucket exchange only
            return orig(bucket, group)
        cur = torch.cuda.current_stream()
        r = {"before": bucket.detach().clone()}
        if path == "device":
            dist.all_reduce(bucket, group=group)
        elif path == "device_sync":
            cur.synchronize()
            dist.all_reduce(bucket, group=group)
        else:
            if path == "emulate":
                ev = torch.cuda.Event()
                ev.record(cur)
                side = torch.cuda.Stream(priority=-1)
                side.wait_event(ev)
                staged = torch.empty(bucket.shape, dtype=bucket.dtype, pin_memory=True)
                with torch.cuda.stream(side):
                    staged.copy_(bucket, non_blocking=True)
                side.synchronize()
                r["staged"] = staged.clone()
            orig(bucket, group)
        r["after"] = bucket.detach().clone()
        torch.cuda.synchronize()
        r["final"] = bucket.detach().cpu().clone()
        r["before"], r["after"] = r["before"].cpu(), r["after"].cpu()
        rec.append(r)
        return world

    vqa_dp.exchange = diag
    import vqvae as VV
    lrec = []
    orig_msl = VV.multispectral_loss_and_grad

    def msl(target, r_, loss_out=None, need_grad=True):
        out = orig_msl(target, r_, loss_out=loss_out, need_grad=need_grad)
        if len(lrec) < 3 and need_grad:  # the first step's three levels
            rec = {"r": r_.detach().clone(), "dr": out[1].detach().clone(), "x": target.x.detach().clone()}
            # the same loss again on the same inputs, in this process (is the spectral kernel chain repeatable
            # while the other rank shares the GPU?), and a checksum of the target spectrograms
            again = orig_msl(target, r_, loss_out=torch.empty(1, device=r_.device), need_grad=True)
            rec["dr_again"] = again[1].detach().clone()
            rec["mags_sum"] = target.mags.view(torch.int32).to(torch.int64).sum().reshape(1)
            lrec.append(rec)
        return out

    VV.multispectral_loss_and_grad = msl
    res = W.run(m, xs, mode)
    torch.cuda.synchronize()
    r_levels = [{k: v.cpu() for k, v in d.items()} for d in lrec]
    r = rec[0]
    r["step1"] = torch.cat([res["step1"]["grads"], res["step1"]["stats"]])
    r["P"] = P
    r["levels"] = r_levels
    r["stats_regions"] = [(int(a), int(b)) for a, b in m.layout["stats"]]
    r["KD"] = (m.vqs[0].num_embeddings if hasattr(m.vqs[0], "num_embeddings") else 0,
               m.vqs[0].embedding_dim if hasattr(m.vqs[0], "embedding_dim") else 0)
    r["offsets"] = {k: (int(o), int(torch.Size(sh).numel())) for k, (o, sh) in m.store.offsets.items()}
    torch.save(r, out)
    dist.barrier()
    dist.destroy_process_group()


REF_LEVELS = []


def reference():
    import vqvae as VV
    refs = []
    orig_msl = VV.multispectral_loss_and_grad
    for r in range(2):
        m = W.build(W.B_LOCAL, config=CONFIG, dtype=DTYPE)
        x = m._as_input(W.batches(2, CONFIG)[0][r * W.B_LOCAL:(r + 1) * W.B_LOCAL])
        lrec = []

        def msl(target, r_, loss_out=None, need_grad=True):
            out = orig_msl(target, r_, loss_out=loss_out, need_grad=need_grad)
            if len(lrec) < 3 and need_grad:
                lrec.append({"r": r_.detach().clone(), "dr": out[1].detach().clone(), "x": target.x.detach().clone(),
                             "mags_sum": target.mags.view(torch.int32).to(torch.int64).sum().reshape(1)})
            return out

        VV.multispectral_loss_and_grad = msl
        m._compute(x, True)
        torch.cuda.synchronize()
        VV.multispectral_loss_and_grad = orig_msl
        REF_LEVELS.append([{k: v.cpu() for k, v in d.items()} for d in lrec])
        refs.append(m.bucket.detach().cpu().clone())
        del m
    torch.cuda.empty_cache()
    return refs


def where(d, offsets, P):
    per = sorted(((float(d[o:o + k].max()), int((d[o:o + k] > 0).sum()), name) for name, (o, k) in offsets.items()),
                 reverse=True)
    per = [f"{nm} {v:.1e}/{c}" for v, c, nm in per if v > 0][:6]
    if float(d[P:].max()) > 0:
        per.append(f"stats/losses {float(d[P:].max()):.1e}/{int((d[P:] > 0).sum())}")
    return per


def main():
    path, reps = sys.argv[1], int(sys.argv[2])
    mode = sys.argv[3] if len(sys.argv) > 3 else "graph"
    refs = reference()
    import tempfile
    out_dir = os.path.join(tempfile.gettempdir(), "dp_diag")  # large: kept out of gpurun_out
    os.makedirs(out_dir, exist_ok=True)
    summary = []
    for rep in range(reps):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        procs, outs = [], []
        for r in range(2):
            out = os.path.join(out_dir, f"{path}_{mode}_rank{r}.pt")
            env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen([sys.executable, __file__, "--worker", path, mode, out], env=env))
            outs.append(out)
        for p in procs:
            assert p.wait(timeout=300) == 0
        rr = [torch.load(o, weights_only=True) for o in outs]
        P = rr[0]["P"]
        want = rr[0]["before"] + rr[1]["before"]
        line = {"path": path, "mode": mode, "rep": rep}
        for r in range(2):
            g = rr[r]
            n_loc = int((g["before"][:P] != refs[r][:P]).sum())
            chk = {"before!=local": n_loc,
                   "after!=sum": int((g["after"] != want).sum()),
                   "final!=sum": int((g["final"] != want).sum()),
                   "final!=after": int((g["final"] != g["after"]).sum()),
                   "step1!=final": int((g["step1"] != g["final"]).sum())}
            # the level statistics at exchange entry (this rank's own m_sumT, n_sum, RT) vs one process: a code
            # count that differs means the argmin (or its input z) differed
            K, D = g["KD"]
            sd = []
            for l, (a, b) in enumerate(g["stats_regions"]):
                got, ref = g["before"][a:b], refs[r][a:b]
                if K and D:
                    n_got, n_ref = got[K * D:K * D + K], ref[K * D:K * D + K]
                    sd.append({"level": l, "m_sum!=": int((got[:K * D] != ref[:K * D]).sum()),
                               "counts!=": int((n_got != n_ref).sum()),
                               "rows_moved": float((n_got - n_ref).abs().sum()) / 2,
                               "RT!=": int((got[K * D + K:] != ref[K * D + K:]).sum())})
            chk["stats"] = sd
            # per level: the reconstruction r, the spectral-loss gradient, the target waveform (rank vs one process)
            lv = []
            for a, b in zip(g["levels"], REF_LEVELS[r]):
                e = dict({k: int((a[k] != b[k]).sum()) for k in b}, dr_repeat=int((a["dr_again"] != a["dr"]).sum()))
                d = (a["r"].double() - b["r"].double()).reshape(a["r"].shape[0], -1)
                if e["r"]:
                    nz = d.nonzero()
                    e["r_maxdiff"] = float(d.abs().max())
                    e["r_maxval"] = float(b["r"].abs().max())
                    e["r_where"] = [(int(i), int(t)) for i, t in nz[:12]]
                lv.append(e)
            chk["levels"] = lv
            if n_loc:
                dl = (g["before"][:P].double() - refs[r][:P].double()).abs()
                chk["before_where"] = where(torch.cat([dl, torch.zeros(g["before"].numel() - P, dtype=dl.dtype)]),
                                            g["offsets"], P)
                # the parameters whose gradient differs, in forward order of the layers (first = most upstream)
                chk["before_params"] = [nm for nm, (o, k) in sorted(g["offsets"].items(), key=lambda t: t[1][0])
                                        if float(dl[o:o + k].max()) > 0][:12]
                # per top-level module: differing / all parameters, and the differing ones in layout order
                groups = {}
                for nm, (o, k) in sorted(g["offsets"].items(), key=lambda t: t[1][0]):
                    top = nm.split("/")[0]
                    dif = float(dl[o:o + k].max()) > 0
                    gr = groups.setdefault(top, [0, 0, []])
                    gr[0] += dif
                    gr[1] += 1
                    if dif:
                        gr[2].append(nm[len(top) + 1:] + f"({float(dl[o:o + k].max()):.0e})")
                chk["groups"] = {t: f"{a}/{b}" for t, (a, b, _) in groups.items()}
                chk["group_params"] = {t: lst for t, (a, b, lst) in groups.items() if a}
            if "staged" in g:
                chk["staged!=before"] = int((g["staged"] != g["before"]).sum())
            if chk["after!=sum"]:
                d = (g["after"].double() - want.double()).abs()
                chk["after_where"] = where(d, g["offsets"], P)
                bad = d > 0
                # is the wrong value this rank's own local value (the other's missing), or the other's?
                chk["after==own_before"] = int((g["after"][bad] == g["before"][bad]).sum())
                chk["after==other_before"] = int((g["after"][bad] == rr[1 - r]["before"][bad]).sum())
            line[f"rank{r}"] = chk
        print(json.dumps(line), flush=True)
        summary.append(line)
    nbad = sum(1 for ln in summary if any(ln[f"rank{r}"]["after!=sum"] or ln[f"rank{r}"]["final!=sum"]
                                          for r in range(2)))
    print(f"SUMMARY path={path} mode={mode}: {nbad} of {reps} runs with a wrong exchanged bucket", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--worker":
        worker(sys.argv[2], sys.argv[3], sys.argv[4])
    else:
        main()
