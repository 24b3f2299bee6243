"""Direct ncclAllReduce on a torch process group's communicator (vqa_dp._Rccl), world size 1 (GPU dev tool)."""
import faulthandler
import os
import sys

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    import vqa_dp
    vqa_dp.FORCE_COLLECTIVE = True
    pg = dist.distributed_c10d._get_default_group()
    be = pg._get_backend(dev)
    print("comm ptr", hex(be._comm_ptr()), flush=True)
    r = vqa_dp.rccl_direct(None, dev)
    print("loaded", r.all_reduce, flush=True)
    x = torch.arange(1000, dtype=torch.float32, device=dev)
    r.run(x, [(0, 500), (500, 1000)])
    torch.cuda.synchronize()
    print("eager ok", float(x.sum()), r.log, flush=True)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            x.mul_(2)
            r.run(x, [(0, 1000)])
            x.add_(1)
    g.replay()
    torch.cuda.synchronize()
    print("graph ok", float(x.sum()), r.log, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
