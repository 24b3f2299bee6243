"""One rank of the prior's data-parallel test (tests/test_gpu_prior_dp.py; not collected by pytest).

Runs Prior.train_step with a torch.distributed process group (gloo, every rank on cuda:0) on its shard of the
global batch — eager, or as two captured hipGraphs around the eager all_reduce — and saves the state.
    python tests/prior_dp_worker.py MODE OUT   (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the environment)
MODE: eager | graph, with the suffixes _cond (upsampler form) and / or _drop (dropout 0.1); VQA_PRIOR_DP_FULL=1:
config 4's full SMALL_PRIOR (ctx 8192, 2048 bins, depth 6).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

N_LOCAL = 1


def cfg():
    """The short form (ctx 256, 64 bins, depth 3), or with VQA_PRIOR_DP_FULL=1 BASELINE config 4's SMALL_PRIOR
    itself (ctx 8192, 2048 bins, depth 6; the bench's leg, prior.py:240-335)."""
    from oracle import prior_ref as P
    if os.environ.get("VQA_PRIOR_DP_FULL") == "1":
        return P.PriorConfig(bins=2048, ctx=8192, width=128, depth=6, heads=2, blocks=4, attn_stacks=1)
    return P.PriorConfig(bins=64, ctx=256, width=128, depth=3, heads=2, blocks=4, attn_stacks=1)


def build(process_group=None, cond=False, drop=False):
    """cond: the upsampler form — level 0 of 2 with ConditionerNet on the level above (Sampler.py:24) and genre
    labels (LabelConditioner), every parameter from the seeded store initialisation. drop: the reference's
    default dropout rate 0.1 (embedding and every residual block's attention output)."""
    from oracle import prior_ref as P
    from prior import Prior
    c = cfg()
    pk = dict(width=c.width, depth=c.depth, heads=c.heads, blocks=c.blocks, attn_stacks=c.attn_stacks,
              drop_out_rate=0.1 if drop else 0.0)
    if cond:
        ck = dict(dilation_factor=3, dilation_cycle=4, residual_width=32, residual_depth=8)
        return Prior(0, [(c.ctx,), (c.ctx // 4,)], c.bins, [3, 2], [2, 2], None, pk, ck, genre_classes=10,
                     dtype="fp32", device="cuda:0", seed=3, process_group=process_group)
    pr = Prior(0, [(c.ctx,)], c.bins, [3], [2], None, pk, None, dtype="fp32", device="cuda:0", seed=3,
               process_group=process_group)
    pr.prior.store.set_values(P.init_params(c, 3))
    return pr


def batches(world, cond=False):
    c = cfg()
    g = torch.Generator().manual_seed(17)
    out = []
    for _ in range(2):
        codes = torch.randint(0, c.bins - 1, (N_LOCAL * world, c.ctx), generator=g)
        if cond:
            out.append((codes, torch.randint(0, c.bins - 1, (N_LOCAL * world, c.ctx // 4), generator=g),
                        torch.randint(0, 10, (N_LOCAL * world,), generator=g)))
        else:
            out.append(codes)
    return out


def shard(x, rank):
    """rows [rank * N_LOCAL, +N_LOCAL) of a batch (a tensor or a tuple of tensors), on the device"""
    if isinstance(x, tuple):
        return tuple(t[rank * N_LOCAL:(rank + 1) * N_LOCAL].cuda() for t in x)
    return x[rank * N_LOCAL:(rank + 1) * N_LOCAL].cuda()


def to_dev(x):
    return tuple(t.cuda() for t in x) if isinstance(x, tuple) else x.cuda()


def snapshot(pr):
    st = pr.prior.store
    return {"weights": st.flat.detach().cpu().clone(), "grads": st.grad[:st.size].detach().cpu().clone(),
            "adam_m": pr.optimizer.m.cpu().clone(), "loss": float(pr.results()["loss"]),
            "accuracy": float(pr.results()["accuracy"]), "batch_input": pr._last_batch_input.cpu().clone()}


def main():
    mode, out = sys.argv[1], sys.argv[2]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cond, drop = "_cond" in mode, "_drop" in mode
    mode = mode.split("_")[0]
    pr = build(dist.group.WORLD, cond, drop)
    xs = [shard(x, rank) for x in batches(world, cond)]
    if mode == "eager":
        pr.train_step(xs[0])
        pr.train_step(xs[1])
    else:  # one eager warm-up step on xs[0] (inside capture), then the captured step replayed on xs[1]
        pr.capture_train_step(xs[0], warmup=1)
        pr.train_step(xs[1])
    torch.cuda.synchronize()
    torch.save(snapshot(pr), out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
