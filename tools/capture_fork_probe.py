"""Which fork / join pattern of a direct ncclAllReduce survives hipGraph capture? (GPU dev tool, world size 1)

origin -> 3 "level" streams (work, then the level's collective, then more work) -> joined into the origin, captured
and replayed. Patterns: the collective on one shared exchange stream forked from each level stream in turn
(temporary events / events kept alive to capture_end), on the level stream itself, or on a per-level stream.
    python tools/capture_fork_probe.py level|perlevel|keep|shared[_torch]      (MASTER_ADDR / MASTER_PORT set)
A `_torch` suffix replaces the ncclAllReduce on the side stream by a plain torch kernel (x.add_(0)): the same fork /
join shape with no RCCL call inside the capture (round-6 verdict item 5).
Measured (round 5, PyTorch 2.10 / ROCm 7.0 / RCCL 2.26.6): "level" captures and replays right; "perlevel", "keep"
and "shared" segfault in capture_end (profiles/r5_dp_overlap.txt).
"""
import faulthandler
import os
import sys

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    pat = sys.argv[1]
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    import vqa_dp
    vqa_dp.FORCE_COLLECTIVE = True
    r = vqa_dp.rccl_direct(None, dev)
    xs = [torch.ones(4096, device=dev) * (l + 1) for l in range(3)]
    lv = [torch.cuda.Stream() for _ in range(3)]
    per = [torch.cuda.Stream() for _ in range(3)]
    shared = torch.cuda.Stream()
    keep = []

    def ev(s):
        e = torch.cuda.Event()
        e.record(s)
        keep.append(e)
        return e

    torch_op = pat.endswith("_torch")
    base = pat[:-len("_torch")] if torch_op else pat

    def launch(x, stream):
        if torch_op:
            with torch.cuda.stream(stream):
                x.add_(0)
            return 0
        return r.all_reduce(x.data_ptr(), x.data_ptr(), x.numel(), 7, 0, r.comm, stream.cuda_stream)

    def coll(l):
        x, cur = xs[l], torch.cuda.current_stream()
        if base == "level":
            rc = launch(x, cur)
        else:
            side = per[l] if base == "perlevel" else shared
            if base == "keep":
                side.wait_event(ev(cur))
            else:
                side.wait_stream(cur)
            rc = launch(x, side)
            if base == "keep":
                cur.wait_event(ev(side))
            else:
                cur.wait_stream(side)
        assert rc == 0

    def step():
        main = torch.cuda.current_stream()
        for s in lv:
            s.wait_stream(main)
        for l in range(3):
            with torch.cuda.stream(lv[l]):
                xs[l].mul_(2)
        prev = None
        for l in range(3):
            with torch.cuda.stream(lv[l]):
                if prev is not None and os.environ.get("PROBE_CHAIN") == "1":
                    torch.cuda.current_stream().wait_event(prev)
                coll(l)
                prev = ev(torch.cuda.current_stream())
                xs[l].add_(1)
        for s in lv:
            main.wait_stream(s)

    step()
    torch.cuda.synchronize()
    dot = os.environ.get("PROBE_DOT")
    g = torch.cuda.CUDAGraph(keep_graph=bool(dot))  # keep the captured hipGraph_t for the dump
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        step()
    print(pat, "captured", flush=True)
    if dot:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipGraphDebugDotPrint.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint]
        raw = g.raw_cuda_graph()
        rc = hip.hipGraphDebugDotPrint(ctypes.c_void_p(raw), os.path.abspath(dot).encode(), 1 << 0 | 1 << 2)
        print("hipGraphDebugDotPrint", rc, os.path.abspath(dot), flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(pat, "ok", [float(x[0]) for x in xs], flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
