"""Does this torch build's gloo all_reduce accept a device (HIP) tensor? Two ranks on cuda:0.
    python tools/probe_gloo_cuda.py            (spawns its two ranks itself)
"""
import os
import socket
import subprocess
import sys


def rank_main():
    import torch
    import torch.distributed as dist
    r = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    x = torch.full((1 << 20,), float(r + 1), device="cuda:0")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        y = x * 2  # produced on a side stream: the collective must be ordered after it
        try:
            dist.all_reduce(y)
            ok = bool((y == 6.0).all())
            print(f"rank {r}: device all_reduce ok={ok}", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"rank {r}: device all_reduce raised {type(e).__name__}: {e}", flush=True)
    torch.cuda.synchronize()
    dist.destroy_process_group()


if __name__ == "__main__":
    if "RANK" in os.environ:
        rank_main()
        sys.exit(0)
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ps = [subprocess.Popen([sys.executable, __file__], env=dict(os.environ, RANK=str(r), WORLD_SIZE="2",
                                                                MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)))
          for r in range(2)]
    sys.exit(max(p.wait(timeout=120) for p in ps))
