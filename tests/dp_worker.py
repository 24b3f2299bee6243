"""One rank of the product data-parallel test (tests/test_gpu_dp.py; not collected by pytest).

Runs VQVAE.train_step with a torch.distributed process group (gloo, every rank on cuda:0) on its shard of
the global batch — eager, or as the two captured hipGraphs around the eager all_reduce — then one
`vqvaes[0](x, training=True)` forward (the EMA on global statistics), and saves the resulting state.
    python tests/dp_worker.py MODE OUT [CONFIG [DTYPE]]   (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set)
CONFIG "cfg1" is BASELINE config 1's architecture; "cfg2_short" is the benched architecture (config 2/3: 3
levels, K = 2048, down_depth [3,2,2], the levels on concurrent streams) on an 8192-frame chunk. The ranks run at the
same time on the one GPU.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-based-music--deep-generative-models_amd"), ROOT]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CONFIGS = {
    "cfg1": dict(input_len=4096, levels=1, latent_dim=64, down_depth=[3], strides=[2], num_embeddings=256,
                 residual_width=32, residual_depth=4, dilation_factor=3),
    "cfg2_short": dict(input_len=8192, levels=3, latent_dim=64, down_depth=[3, 2, 2], strides=[2, 2, 2],
                       num_embeddings=2048, residual_width=32, residual_depth=4, dilation_factor=3),
    # BASELINE config 3's per-rank workload: config 2 at its full chunk length (run with VQA_DP_BATCH=32)
    "cfg2": dict(input_len=65536, levels=3, latent_dim=64, down_depth=[3, 2, 2], strides=[2, 2, 2],
                 num_embeddings=2048, residual_width=32, residual_depth=4, dilation_factor=3),
}
CFG = CONFIGS["cfg1"]
B_LOCAL = int(os.environ.get("VQA_DP_BATCH", "2"))  # items per rank
# "all": step 1, step 2, forward-only EMA call; "step1": the first step only (full-size runs)
PHASES = os.environ.get("VQA_DP_PHASES", "all")


def build(B, process_group=None, config="cfg1", dtype="fp32"):
    from oracle import vqvae_ref as R
    from vqvae import VQVAE
    cfg = R.RefConfig(**CONFIGS[config])
    m = VQVAE((cfg.input_len, 1), cfg.levels, cfg.latent_dim, cfg.down_depth, cfg.strides,
              num_embeddings=cfg.num_embeddings, residual_width=cfg.residual_width,
              residual_depth=cfg.residual_depth, dilation_factor=cfg.dilation_factor, dtype=dtype,
              device="cuda:0", process_group=process_group)
    m.set_weights(R.init_params(cfg, 1))
    m.set_vq_state(R.init_vq_state(cfg, 2))
    m.compile()
    return m


def batches(world, config="cfg1"):
    from oracle import vqvae_ref as R
    return [R.synthetic_batch(B_LOCAL * world, CONFIGS[config]["input_len"], seed=90 + i) for i in range(3)]


def snapshot(m):
    P = m.layout["grads"][1]
    return {"weights": m.store.flat.detach().cpu().clone(), "adam_m": m.optimizer.m.cpu().clone(),
            "adam_v": m.optimizer.v.cpu().clone(), "stats": m.bucket[P:].detach().cpu().clone(),
            "grads": m.bucket[:P].detach().cpu().clone(),
            "vq": [{k: torch.as_tensor(v) for k, v in st.items() if k != "calls"} | {"calls": st["calls"]}
                   for st in m.get_vq_state()],
            "results": {k: float(v) for k, v in m.results().items()},
            "offsets": {k: (int(o), int(torch.Size(sh).numel())) for k, (o, sh) in m.store.offsets.items()}}


def run(m, xs, mode):
    """The sequence both the ranks and the single-process reference execute: step on xs[0], step on xs[1]
    (eager, or: capture = one eager warm-up step on xs[0], then the captured step replayed on xs[1]), then
    one forward-only EMA call of level 0 on xs[2]. Snapshots after the first step, the second step and the
    forward."""
    res = {}
    if mode == "eager":
        m.train_step(xs[0])
        torch.cuda.synchronize()
        res["step1"] = snapshot(m)
        if PHASES == "step1":
            return res
        m.train_step(xs[1])
    else:
        m.capture_train_step(xs[0], warmup=1)
        torch.cuda.synchronize()
        res["step1"] = snapshot(m)
        if PHASES == "step1":
            return res
        if PHASES == "mixed":
            # an eager test_step between the capture and the next replay: the replay must still exchange the
            # whole bucket the captured graphs were split around, whatever form the eager step used
            m.test_step(xs[2])
            torch.cuda.synchronize()
            res["test"] = snapshot(m)
        m.train_step(xs[1])
    torch.cuda.synchronize()
    res["steps"] = snapshot(m)
    m.vqvaes[0](xs[2], training=True)  # forward-only EMA: global statistics under DP
    torch.cuda.synchronize()
    res["forward"] = snapshot(m)
    return res


def main():
    mode, out = sys.argv[1], sys.argv[2]
    config = sys.argv[3] if len(sys.argv) > 3 else "cfg1"
    dtype = sys.argv[4] if len(sys.argv) > 4 else "fp32"
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = build(B_LOCAL, config=config, dtype=dtype)
    xs = [x[rank * B_LOCAL:(rank + 1) * B_LOCAL] for x in batches(world, config)]
    local, post = [], []
    if os.environ.get("VQA_DP_PROBE") == "1":
        # the exchange's stream contract, both sides, as device copies queued IN ORDER on the current stream
        # (no host sync): at entry the bucket holds this rank's complete local gradient (what RCCL reads), and
        # right after `exchange` returns it holds the sum over ranks (what `_update` / the second graph reads)
        import vqa_dp
        P = m.layout["grads"][1]
        exchange = vqa_dp.exchange

        def probe(bucket, group=None):
            full = bucket.numel() > P
            if full:
                local.append(bucket[:P].detach().clone())
            w = exchange(bucket, group)
            if full:
                post.append(bucket[:P].detach().clone())
            return w

        vqa_dp.exchange = probe
    res = run(m, xs, mode)
    if local:
        res["local_step1"] = local[0].cpu()
        res["post_step1"] = post[0].cpu()
    torch.save(res, out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
