"""The RCCL branch of the data-parallel step on ONE GPU (tests/test_gpu_rccl.py; not collected by pytest).

A world-size-1 "nccl" process group (RCCL) with vqa_dp.FORCE_COLLECTIVE: the step takes its DP path — the EMA after
the exchange, `dist.all_reduce` of the device bucket on the producer stream, two hipGraphs around it — and must end
bitwise where the same model without the DP path ends (a one-rank sum is the bucket itself).
    python tests/rccl_worker.py OUT [overlap]   (MASTER_ADDR / MASTER_PORT set; NCCL_DEBUG=INFO shows RCCL's own log)
"overlap": the DP runs with VQVAE.overlap_exchange — one collective per level region on the level's stream and the
losses after the join, captured with the step into ONE graph.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT, HERE]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import dp_worker as W  # noqa: E402


def main():
    out = sys.argv[1]
    overlap = len(sys.argv) > 2 and sys.argv[2] == "overlap"
    os.environ["VQA_DP_OVERLAP"] = "1" if overlap else "0"
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    import vqa_dp
    calls = []
    orig = dist.all_reduce

    def counted(t, *a, **k):
        calls.append({"device": str(t.device), "numel": int(t.numel()), "backend": str(dist.get_backend())})
        return orig(t, *a, **k)

    dist.all_reduce = counted
    W.B_LOCAL = 2
    xs = W.batches(1, "cfg2_short")
    res = {}
    for mode in ("eager", "graph"):
        for forced in (False, True):
            vqa_dp.FORCE_COLLECTIVE = forced
            n0 = len(calls)
            m = W.build(2, config="cfg2_short", dtype="bf16")
            if mode == "eager":
                m.train_step(xs[0])
                m.train_step(xs[1])
            else:
                m.capture_train_step(xs[0], warmup=1)  # one eager warm-up step on a side stream, then the graphs
                m.train_step(xs[1])
                m.train_step(xs[2])
                assert (m._graph[1] is not None) == (forced and not overlap), "split graphs exactly on the one-bucket DP path"
            torch.cuda.synchronize()
            snap = W.snapshot(m)
            snap["all_reduce_calls"] = calls[n0:]
            direct = [r.log for r in vqa_dp._RCCL.values()]
            snap["direct_calls"] = [n for lg in direct for n in lg]
            for lg in direct:
                lg.clear()
            snap["regions"] = [[list(r) for r in regs] for regs in m.level_regions] + [list(m.layout["losses"])]
            res[f"{mode}_{'dp' if forced else 'single'}"] = snap
            del m
            torch.cuda.empty_cache()
    vqa_dp.FORCE_COLLECTIVE = False
    torch.save(res, out)
    vqa_dp.reset()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
