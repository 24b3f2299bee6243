"""Does torch-gloo's all_reduce of a DEVICE tensor read it in order after the caller's current stream? (GPU dev tool)

Two gloo ranks on cuda:0. Each rank makes the value it contributes on a stream after a long spin kernel
(torch.cuda._sleep), then calls dist.all_reduce on the device tensor with no host sync, and checks the sum once
everything has finished. Cases:
  default     current stream = the default stream
  side        current stream = a side stream (as capture_train_step's warm-up runs the VQ-VAE step)
  side_join   the value is produced on another stream that the side stream joined (wait_stream), as the
              levels' streams join the producer stream
  side_sync   like side, with hipStreamSynchronize of the current stream before the all_reduce
  side_host   like side, through the product's vqa_dp.exchange (host staging on the current stream)
  side_join3  the step's topology: three producer streams (the levels), each writing its third of the tensor
              behind a spin of a different length, all joined into the side stream; more streams than the
              box's 4 hardware queues are alive (the levels', the side stream, gloo's pool stream, the default)
Prints one line per case: the sum (want 2 * world... = 3.0 with values 1 and 2) and the stale value if the
staging copy ran before the producer finished.

    python tools/gloo_stream_probe.py [spin_cycles]
"""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]


def run(rank, world, port, cycles, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import vqa_dp
    out = {}
    levels = [torch.cuda.Stream() for _ in range(3)]
    for case in ("default", "side", "side_join", "side_sync", "side_host", "side_join3", "side_join3", "default",
                 "side"):
        t = torch.zeros(1 << 20, device="cuda")  # 4 MB, stale value 0
        torch.cuda.synchronize()
        dist.barrier()
        s = torch.cuda.Stream() if case != "default" else torch.cuda.current_stream()
        other = torch.cuda.Stream()
        with torch.cuda.stream(s):
            if case == "side_join3":
                n3 = t.numel() // 3
                for i, ls in enumerate(levels):
                    ls.wait_stream(s)
                    with torch.cuda.stream(ls):
                        torch.cuda._sleep(cycles // (3 - i))
                        t[i * n3:(i + 1) * n3 if i < 2 else t.numel()].fill_(rank + 1.0)
                for ls in levels:
                    s.wait_stream(ls)
            elif case == "side_join":
                other.wait_stream(s)
                with torch.cuda.stream(other):
                    torch.cuda._sleep(cycles)
                    t.fill_(rank + 1.0)
                s.wait_stream(other)
            else:
                torch.cuda._sleep(cycles)
                t.fill_(rank + 1.0)
            if case == "side_sync":
                s.synchronize()
            if case == "side_host":
                vqa_dp.exchange(t)
            else:
                dist.all_reduce(t)
            after = t.clone()  # the consumer's view, queued on the current stream
        torch.cuda.synchronize()
        vals = sorted(set(after.cpu().tolist()))
        key = case if case not in out else case + "_again"
        out[key] = vals
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def main():
    cycles = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000_000
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=run, args=(r, 2, port, cycles, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
    print(f"torch {torch.__version__}, spin {cycles} cycles before the producer's write; want [3.0]")
    for k, v in out.items():
        print(f"  {k:16s} sum values seen: {v}  {'OK' if v == [3.0] else 'STALE (the collective read before the producer finished)'}")


if __name__ == "__main__":
    main()
