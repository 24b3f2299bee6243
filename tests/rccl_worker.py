"""The RCCL branch of the data-parallel step on ONE GPU (tests/test_gpu_rccl.py; not collected by pytest).

A world-size-1 "nccl" process group (RCCL) with vqa_dp.FORCE_COLLECTIVE: the step takes its DP path — the EMA after
the exchange, `dist.all_reduce` of the device bucket on the producer stream, two hipGraphs around it — and must end
bitwise where the same model without the DP path ends (a one-rank sum is the bucket itself).
    python tests/rccl_worker.py OUT      (MASTER_ADDR / MASTER_PORT set; NCCL_DEBUG=INFO shows RCCL's own log)
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
                assert (m._graph[1] is not None) == forced, "split graphs exactly on the DP path"
            torch.cuda.synchronize()
            snap = W.snapshot(m)
            snap["all_reduce_calls"] = calls[n0:]
            res[f"{mode}_{'dp' if forced else 'single'}"] = snap
            del m
            torch.cuda.empty_cache()
    vqa_dp.FORCE_COLLECTIVE = False
    torch.save(res, out)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
