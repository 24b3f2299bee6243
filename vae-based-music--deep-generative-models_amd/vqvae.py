"""Multi-level VQ-VAE — drop-in for the reference vqvae.py (VQVAE, get_vqvae).

vqvae.py:30-91    VQVAE(input_shape, levels, latent_dim, down_depth, strides, num_embeddings=128,
                  residual_width=64, residual_depth=4, dilation_factor=1, train_variance=1.0): `levels`
                  independent {Encoder(depth=l+1), VectorQuantizer, Decoder(depth=l+1)} on the waveform.
vqvae.py:111-146  train_step: per level recon MSE + commitment + multispectral loss, summed; gradients of
                  all levels' conv weights; Adam.
vqvae.py:148-172  test_step (the VQ keeps its default training=True, so the EMA runs — kept on purpose).
vqvae.py:178-206  call(x, training=False) -> (recons, loss lists).
vqvae.py:208-260  encode / encode_level / decode / decode_level.
vqvae.py:262-304  update_metrics (running means; key names kept).

MI355X design: every conv / VQ / loss / optimizer op is a libvqa HIP kernel called through the C-ABI on
torch's current stream; the backward is written out explicitly (no autograd tape over the conv stack);
each level runs forward then backward immediately (levels are independent), so only one level's
activations are alive. Weights, gradients and the codebook EMA sums are flat fp32 buffers: the whole
data-parallel exchange sums [grads | EMA sums | reset rows | losses] over ranks: on RCCL per level as soon as that
level's backward ends (`overlap_exchange`, vqa_dp.level_regions) or as ONE all_reduce after the join (default).
`capture_train_step` records the full step as a hipGraph (torch.cuda.graph) so replay has no host cost.
"""
from __future__ import annotations

import os
from itertools import chain
from typing import Dict, List, Optional

import numpy as np
import torch

import vqa_dp
import vqa_lib as V
from data_utils import SpectralTarget, multispectral_loss_and_grad
from encdec import Decoder, Encoder
from vqa_layers import CKPT_VERSION, ParamStore, checkpoint_layout
from vqa_metrics import SlotMean
from vqa_module import keras_evaluate
from vqa_optim import Adam
from VectorQuantizer import VectorQuantizer


def _dtype(d) -> torch.dtype:
    if d in ("bf16", "bfloat16", torch.bfloat16):
        return torch.bfloat16
    if d in ("fp32", "float32", torch.float32):
        return torch.float32
    raise ValueError(f"unsupported compute dtype {d}")


class LevelModel:
    """The per-level keras.Model of get_vqvae (vqvae.py:15-21): x -> encoder -> vq -> decoder on an input of
    fixed shape `input_shape` (keras.Input). Inside a VQVAE it runs on the model's kernels and buffers
    (`vqvaes[level]`); from get_vqvae it owns a parameter store of its own."""

    def __init__(self, input_shape, encoder, decoder, vq, level=0, owner: Optional["VQVAE"] = None,
                 dtype="fp32", device=None, seed=1):
        self.input_shape = tuple(input_shape)
        self.encoder, self.decoder, self.vq, self.level, self.owner = encoder, decoder, vq, level, owner
        self.name = f"vq_vae_{level}"
        if owner is None:
            self.cdt = _dtype(dtype)
            self.device = torch.device(device) if device is not None else vq.device
            self.store = ParamStore()
            if not encoder.built:
                encoder.build(self.store, f"enc{level}", int(self.input_shape[-1]), self.cdt)
            if not decoder.built:
                decoder.build(self.store, f"dec{level}", vq.embedding_dim, self.cdt)
            self.store.materialize(self.device, seed=seed)

    def __call__(self, x, training=True):
        if self.owner is not None:
            return self.owner._level_forward_only(self.owner._as_input(x), self.level, training)
        x = x[0] if isinstance(x, (tuple, list)) else x
        x = torch.as_tensor(x).to(device=self.device, dtype=torch.float32)
        if x.dim() == 2:
            x = x.unsqueeze(-1)
        if tuple(x.shape[1:]) != self.input_shape:
            raise ValueError(f"input shape {tuple(x.shape)} does not match keras.Input{self.input_shape}")
        with torch.no_grad():
            z = self.encoder.forward(x.contiguous())
            q, _ = self.vq.call(z, training=training)
            return self.decoder.forward(q)

    call = __call__

    @property
    def losses(self):
        return self.vq.losses

    @property
    def trainable_variables(self):
        st = self.owner.store if self.owner is not None else self.store
        pre = (f"enc{self.level}/", f"dec{self.level}/")
        return [st.view(n) for n, _, _ in st.specs if n.startswith(pre)]


def get_vqvae(input_shape, encoder, decoder, vq, level=0, **kwargs):
    """vqvae.py:15-21 — the single-level model x -> encoder -> vq -> decoder (keras default init of the
    encoder / decoder weights unless they are already built)."""
    return LevelModel(input_shape, encoder, decoder, vq, level, **kwargs)


class VQVAE:
    def __init__(self, input_shape, levels, latent_dim, down_depth, strides, num_embeddings=128, residual_width=64,
                 residual_depth=4, dilation_factor=1, train_variance=1.0, *, dtype="bf16", device="cuda",
                 seed=1, codebook_seed=2, reset_seed=3, process_group=None, name="vqvae", overlap_exchange=None,
                 **kwargs):
        self.input_shape = tuple(input_shape)
        self.T = int(self.input_shape[0])
        self.channels = int(self.input_shape[-1]) if len(self.input_shape) > 1 else 1
        self.levels = levels
        self.train_variance = train_variance
        self.latent_dim = latent_dim
        self.num_embeddings = num_embeddings
        self.down_depth, self.strides = list(down_depth), list(strides)
        self.cdt = _dtype(dtype)
        self.device = torch.device(device)
        self.name = name
        self.process_group = process_group
        # data-parallel exchange per level, overlapped with the other levels' chains (vqa_dp): True / False, or None =
        # VQA_DP_OVERLAP=1 (off by default: the multi-rank captured form has not run on hardware)
        self._overlap_cfg = bool(overlap_exchange) if overlap_exchange is not None else (
            os.environ.get("VQA_DP_OVERLAP", "0") == "1")
        # the order the levels' exchanges are issued in (one communicator: its collectives run in issue order, so
        # the level whose chain ends first goes first; VQA_DP_OVERLAP_ORDER="0,1,2")
        self.exchange_order = [int(v) for v in os.environ.get("VQA_DP_OVERLAP_ORDER", ",".join(
            str(l) for l in range(levels))).split(",")]
        assert sorted(self.exchange_order) == list(range(levels)), self.exchange_order

        self.vqs = [VectorQuantizer(num_embeddings, latent_dim, level=l, name=f"vector_quantizer_{l}",
                                    device=self.device, seed=codebook_seed + 1000 * l, reset_seed=reset_seed)
                    for l in range(levels)]
        self.encoders = [Encoder(output_dim=latent_dim, residual_width=residual_width, residual_depth=residual_depth,
                                 depth=l + 1, down_depth=self.down_depth[:l + 1], strides=self.strides[:l + 1],
                                 dilation_factor=dilation_factor, name=f"encoder_{l}") for l in range(levels)]
        self.decoders = [Decoder(output_dim=self.channels, embed_width=latent_dim, residual_width=residual_width,
                                 residual_depth=residual_depth, depth=l + 1, down_depth=self.down_depth[:l + 1],
                                 strides=self.strides[:l + 1], dilation_factor=dilation_factor, name=f"decoder_{l}")
                         for l in range(levels)]
        self.store = ParamStore()
        for l in range(levels):
            d = self.encoders[l].build(self.store, f"enc{l}", self.channels, self.cdt)
            assert d == latent_dim
            self.decoders[l].build(self.store, f"dec{l}", latent_dim, self.cdt)
        self.latent_lens = []
        for l in range(levels):
            t = self.T
            for b in range(l + 1):
                for _ in range(self.down_depth[b]):
                    t = -(-t // self.strides[b])
            self.latent_lens.append(t)
        self.hops = [self.T // t for t in self.latent_lens]  # 8 / 32 / 128 at down_depth [3,2,2] (vqvae.py:54)

        # all-reduce bucket: [grads (P, padded) | per-level VQ stats | per-level (recon, commit, spectral)]
        lay = vqa_dp.bucket_layout(self.store.size, [vq.stats_size() for vq in self.vqs], levels)
        self.layout = lay
        P = lay["grads"][1]
        self.bucket = torch.zeros(lay["total"], dtype=torch.float32, device=self.device)
        self.store.materialize(self.device, grad_buffer=self.bucket[:P], seed=seed)
        for vq, (a, b) in zip(self.vqs, lay["stats"]):
            vq.bind_stats(self.bucket[a:b])
        self._stats_region = self.bucket[P:]
        self.loss_slots = self.bucket[lay["losses"][0]:lay["losses"][1]].view(levels, 3)
        self._loss_region = [tuple(lay["losses"])]
        # each level's slices of the bucket: its layers' gradient range (enc{l}/*, dec{l}/*) and its VQ statistics
        self.level_regions = vqa_dp.level_regions(lay, vqa_dp.level_param_ranges(self.store.offsets, levels))
        self._overlapped = False  # did the last _compute exchange per level (then _exchange sums the losses only)
        self._exchange_events: List[torch.cuda.Event] = []
        for l, vq in enumerate(self.vqs):
            vq.commit = self.loss_slots[l, 1:2]

        # metric trackers (vqvae.py:77-89 + VectorQuantizer.py:62-64): ONE device accumulator, rows in the
        # order of the returned dict (update_metrics, vqvae.py:262-304), updated by one vqa_step_metrics launch
        names = ["loss", "recon_loss", "vqvae_loss", "spectral_loss"]
        for l in range(levels):
            names += [f"[{l}]level_loss", f"[{l}]recon_loss", f"[{l}]vq_loss", f"[{l}]spectral_loss",
                      f"[{l}]batch_codebook_usage", f"[{l}]codebook_usage", f"[{l}]codebook_entropy"]
        self.metric_names = names
        self._macc = torch.zeros(len(names), 2, dtype=torch.float32, device=self.device)
        self._vq_metrics = torch.zeros(levels, 3, dtype=torch.float32, device=self.device)
        row = {n: i for i, n in enumerate(names)}
        # keras.metrics.Mean trackers with the reference's names (vqvae.py:78-89), views of _macc rows
        self.total_loss_tracker = SlotMean("total_loss", self._macc, row["loss"])
        self.reconstruction_loss_tracker = SlotMean("reconstruction_loss", self._macc, row["recon_loss"])
        self.vq_loss_tracker = SlotMean("vq_loss", self._macc, row["vqvae_loss"])
        self.spectral_loss_tracker = SlotMean("spectral_loss", self._macc, row["spectral_loss"])
        self.level_loss_trackers, self.recon_loss_trackers, self.vq_loss_trackers, self.spectral_loss_trackers = (
            [SlotMean(f"[{l}]{k}", self._macc, row[f"[{l}]{k}"]) for l in range(levels)]
            for k in ("level_loss", "recon_loss", "vq_loss", "spectral_loss"))
        for l, vq in enumerate(self.vqs):
            vq.bind_metrics(self._vq_metrics[l], self._macc,
                            [row[f"[{l}]{k}"] for k in ("batch_codebook_usage", "codebook_usage", "codebook_entropy")])
        self.optimizer: Optional[Adam] = None
        self.vqvaes = [LevelModel(self.input_shape, self.encoders[l], self.decoders[l], self.vqs[l], l, owner=self)
                       for l in range(levels)]
        self._graph = None
        # run the levels' independent forward/backward chains on one stream each (VQA_LEVEL_STREAMS=0: serial)
        self.concurrent_levels = os.environ.get("VQA_LEVEL_STREAMS", "1") != "0"
        self._streams = None
        # A/B switch (VQA_STEP_LAYOUT=r3): the round-3 step layout — the target spectrograms on the producer stream
        # before the levels fork, every level's codebook EMA after the join
        self._r3_layout = os.environ.get("VQA_STEP_LAYOUT") == "r3"

    # ------------------------------------------------------------------ keras-like API
    def compile(self, optimizer=None, **kwargs):
        """keras Model.compile: a vqa_optim.Adam (float or LearningRateSchedule learning rate). A captured step
        is dropped: it holds the previous optimizer's buffers (m, v, step counter, learning rate)."""
        self.optimizer = optimizer or Adam()
        self.optimizer.build(self.store)
        self._graph = None
        self._graph_pool = None

    @property
    def metrics(self):
        """vqvae.py:93-104: the model's keras Mean trackers (total, reconstruction, vq, spectral, then the
        per-level level / recon / vq / spectral trackers). `for m in model.metrics: m.reset_state()`
        (src/callback/vae_monitor.py:64-65) and `m.name`, `m.result()` (:71) work unchanged."""
        return [self.total_loss_tracker, self.reconstruction_loss_tracker, self.vq_loss_tracker,
                self.spectral_loss_tracker, *self.level_loss_trackers, *self.recon_loss_trackers,
                *self.vq_loss_trackers, *self.spectral_loss_trackers]

    def reset_metrics(self):
        """keras Model.reset_metrics: resets `self.metrics` only. The codebook usage / entropy trackers are
        not in that list (VectorQuantizer.metrics), so, as in the reference, they keep accumulating."""
        for m in self.metrics:
            m.reset_state()

    def get_quantizer(self):
        return self.vqs[0]

    def _as_input(self, data) -> torch.Tensor:
        x = data[0] if isinstance(data, (tuple, list)) else data
        x = torch.as_tensor(x) if not isinstance(x, torch.Tensor) else x
        x = x.to(device=self.device, dtype=torch.float32)
        if x.dim() == 2:
            x = x.unsqueeze(-1)
        if tuple(x.shape[1:]) != (self.T, self.channels):
            raise ValueError(f"input shape {tuple(x.shape)} does not match keras.Input{(self.T, self.channels)}")
        return x.contiguous()

    def _world(self) -> int:
        return vqa_dp.world_size(self.process_group)

    def _rank(self) -> int:
        return vqa_dp.rank(self.process_group)

    # ------------------------------------------------------------------ the step
    def _compute(self, x: torch.Tensor, training_grads: bool):
        """Forward (+ backward when training_grads) of every level; EMA sums into the bucket. On one device the
        codebook EMA of each level runs at the end of its own chain (only the bucket exchange needs it later)."""
        self._stats_region.zero_()
        main = torch.cuda.current_stream(self.device)
        streams = self._level_streams()
        overlap = self._overlap_now()
        self._overlapped = overlap
        self._exchange_events = []
        ema_in_level = not vqa_dp.active(self.process_group) and not self._r3_layout
        if streams is None or self._r3_layout:
            target = SpectralTarget(x)
        if streams is None:
            for l in range(self.levels):
                self._level_step(x, l, target, training_grads, ema_in_level)
                if overlap:
                    self._level_exchange(l, training_grads)
        else:
            for s in streams:
                s.wait_stream(main)
            # the target spectrograms (needed only by each level's loss) on level 0's stream, the shortest chain:
            # the longer levels start their encoders at once and wait for the target at their losses
            if not self._r3_layout:
                with torch.cuda.stream(streams[0]):
                    target = SpectralTarget(x)
            for l in range(self.levels):
                with torch.cuda.stream(streams[l]):
                    self._level_step(x, l, target, training_grads, ema_in_level)
            if overlap:
                # every chain is queued before the first collective (a host-staged gloo exchange blocks the host);
                # each level's collectives wait for the previous level's (an event, not a join of the chains), so
                # they execute in one order on every rank whatever RCCL does with collectives on concurrent streams
                prev = None
                for l in self.exchange_order:
                    with torch.cuda.stream(streams[l]):
                        prev = self._level_exchange(l, training_grads, after=prev)
            for s in streams:
                main.wait_stream(s)
        self.store.deferred = None

    @property
    def overlap_exchange(self) -> bool:
        return self._overlap_cfg

    def _overlap_now(self) -> bool:
        """Exchange per level in this _compute? Only on the data-parallel path, and not while a host-staged (gloo)
        exchange would have to be captured into a graph (capture_train_step then keeps the split graphs)."""
        if not (self.overlap_exchange and vqa_dp.active(self.process_group)) or self._r3_layout:
            return False
        return not (self.device.type == "cuda" and torch.cuda.is_current_stream_capturing()
                    and vqa_dp.host_staged(self.bucket, self.process_group))

    def _level_exchange(self, l: int, grads: bool, after: Optional[torch.cuda.Event] = None):
        """Level l's share of the exchange on the current (level) stream — after the event `after` (the previous
        level's collectives) — then its codebook EMA on the sums. Returns the event that follows its collectives."""
        cur = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        if after is not None:
            cur.wait_event(after)
        g, st = self.level_regions[l]
        vqa_dp.exchange_regions(self.bucket, [g, st] if grads else [st], self.process_group)
        done = None
        if cur is not None:
            done = torch.cuda.Event()
            done.record(cur)
            self._exchange_events.append(done)  # alive until the next step's exchange (capture_end reads them)
        self.vqs[l].apply_ema(update_trackers=False)
        return done

    def _level_streams(self):
        """One HIP stream per level when `concurrent_levels`: the levels share nothing but the input and
        its spectrograms, so their kernel chains overlap (level 2's long tail of small, latency-bound
        launches fills the gaps of level 0's HBM-bound ones). Every buffer a level writes is its own (its
        layers' gradient slices, its VQ stats and loss slots, workspaces from its stream's pool)."""
        if not self.concurrent_levels or self.device.type != "cuda":
            return None
        if self._streams is None:
            self._streams = [torch.cuda.Stream(device=self.device) for _ in range(self.levels)]
        return self._streams

    def _level_step(self, x, l, target, training_grads, ema=False):
        # this level's weight-gradient partials are reduced in one launch at its end
        self.store.deferred = V.Deferred() if training_grads else None
        enc, vq, dec = self.encoders[l], self.vqs[l], self.decoders[l]
        z = enc.forward(x, save=training_grads)
        n_loc = z.shape[0] * z.shape[1]
        row_offset, n_global = vqa_dp.global_row_range(n_loc, self.process_group)
        q, _ = vq.forward(z, training=True, row_offset=row_offset, n_global=n_global, save=training_grads)
        r = dec.forward(q, save=training_grads)
        _, dr_spec = multispectral_loss_and_grad(target, r, loss_out=self.loss_slots[l, 2:3],
                                                 need_grad=training_grads)
        dr = torch.empty_like(r)
        V.mse_loss(x, r, dr_spec, dr, self.loss_slots[l, 0:1])
        if training_grads:
            dq = dec.backward(dr)
            dz = vq.backward(dq, n_global=n_loc)  # reads the codebook this step quantised with
            enc.backward(dz)
            self.store.deferred.flush()
        if ema:
            vq.apply_ema(update_trackers=False)  # after every use of the old codebook in this level

    def _update(self, apply_grads: bool):
        world = self._world()
        if apply_grads:
            self.optimizer.apply(self.store, grad_scale=1.0 / world)
        if (vqa_dp.active(self.process_group) and not self._overlapped) or self._r3_layout:
            # else the levels' chains applied it (_compute)
            for vq in self.vqs:
                vq.apply_ema(update_trackers=False)
        # update_metrics (vqvae.py:262-304) + the VQ trackers: one launch
        V.step_metrics(self.loss_slots, self._vq_metrics, self._macc, self.levels, 1.0 / world)

    def _exchange(self, grads: bool = True):
        """The step's one collective: all_reduce(SUM) of [grads | EMA sums | reset rows | losses]; without
        gradients (test_step) only the statistics region. After an overlapped _compute only the losses are left."""
        if self._overlapped:
            vqa_dp.exchange_regions(self.bucket, self._loss_region, self.process_group)
            return
        vqa_dp.exchange(self.bucket if grads else self._stats_region, self.process_group)

    def update_metrics(self, level_losses, recon_losses, commit_losses, spectral_losses):
        """vqvae.py:262-304 for externally computed per-level losses (the step itself updates the same
        trackers in one launch, vqa_step_metrics): the total / recon / vq / spectral trackers take the sums over
        levels, each level's trackers its own values; returns the reference's dict (the four totals, then per
        level its trackers and its VectorQuantizer's)."""
        def val(v):
            return torch.as_tensor(v, dtype=torch.float32, device=self.device).reshape(())
        lv, rv, cv, sv = ([val(v) for v in vs] for vs in (level_losses, recon_losses, commit_losses, spectral_losses))
        self.total_loss_tracker.update_state(sum(lv))
        self.reconstruction_loss_tracker.update_state(sum(rv))
        self.vq_loss_tracker.update_state(sum(cv))
        self.spectral_loss_tracker.update_state(sum(sv))
        out = {"loss": self.total_loss_tracker.result(), "recon_loss": self.reconstruction_loss_tracker.result(),
               "vqvae_loss": self.vq_loss_tracker.result(), "spectral_loss": self.spectral_loss_tracker.result()}
        for l in range(self.levels):
            for trackers, v in ((self.level_loss_trackers, lv), (self.recon_loss_trackers, rv),
                                (self.vq_loss_trackers, cv), (self.spectral_loss_trackers, sv)):
                trackers[l].update_state(v[l])
                out[trackers[l].name] = trackers[l].result()
            out.update({m.name: m.result() for m in self.vqs[l].metrics})
        return out

    def _multispectral_loss(self, x, reconstructions):
        """vqvae.py:309-326: the multi-resolution spectral loss of `reconstructions` against `x` — the batch mean,
        as a 0-dim device tensor (the reference's callers take tf.reduce_mean of it, which leaves it unchanged)."""
        x = self._as_input(x)
        r = torch.as_tensor(reconstructions, device=self.device).float().reshape(x.shape).contiguous()
        loss, _ = multispectral_loss_and_grad(SpectralTarget(x), r, need_grad=False)
        return loss.reshape(())

    def results(self) -> Dict[str, torch.Tensor]:
        res = self._macc[:, 0] / self._macc[:, 1].clamp(min=1.0)
        return {n: res[i] for i, n in enumerate(self.metric_names)}

    def train_step(self, data):
        """vqvae.py:111-146. Returns the running-mean metric dict (0-dim device tensors)."""
        if self.optimizer is None:
            self.compile()
        x = self._as_input(data)
        if self._graph is not None and x.shape == self._graph_x.shape:
            self._graph_x.copy_(x)
            self._replay()
            return self.results()
        self._compute(x, training_grads=True)
        self._exchange()
        self._update(apply_grads=True)
        return self.results()

    def test_step(self, data):
        """vqvae.py:148-172 — forward + losses; the VQ EMA runs (reference default training=True)."""
        x = self._as_input(data)
        with torch.no_grad():
            self._compute(x, training_grads=False)
            self._exchange(grads=False)
            self._update(apply_grads=False)
        return self.results()

    def evaluate(self, x=None, y=None, batch_size=None, verbose=0, steps=None, return_dict=False, **kwargs):
        """keras Model.evaluate over test_step (vqvae.py:148-172), as src/callback/vae_monitor.py:69 calls it on
        the validation dataset: metrics reset, test_step per batch (the codebook EMA runs, VectorQuantizer.py:75),
        the running means returned (vqa_module.keras_evaluate)."""
        return keras_evaluate(self, x, y, batch_size=batch_size, verbose=verbose, steps=steps,
                              return_dict=return_dict)

    # ------------------------------------------------------------------ hipGraph capture
    def capture_train_step(self, x_example, warmup: int = 2):
        """Run `warmup` eager steps (real steps) then record one full train step as a hipGraph; later
        train_step calls with this batch shape copy the batch in and replay. With a process group the
        step is two graphs around the eager RCCL all_reduce; with `overlap_exchange` on a device-side backend
        (RCCL) the per-level collectives are captured with the step into one graph."""
        if self.optimizer is None:
            self.compile()
        x = self._as_input(x_example)
        self._graph_x = x.clone()
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._compute(self._graph_x, True)
                self._exchange()
                self._update(True)
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        if self.overlap_exchange and vqa_dp.active(self.process_group) and vqa_dp.device_side(self.process_group):
            # the direct-RCCL issuer (and, if the group made it lazily, its communicator) exists before the capture
            vqa_dp.rccl_direct(self.process_group, self.device)
        self._graph_pool = torch.cuda.graph_pool_handle()
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1, pool=self._graph_pool, capture_error_mode="thread_local"):
            self._compute(self._graph_x, True)
            one_graph = self._overlapped or not vqa_dp.active(self.process_group)
            if self._overlapped:
                self._exchange()
            if one_graph:
                self._update(True)
        g2 = None
        if not one_graph:
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, pool=self._graph_pool, capture_error_mode="thread_local"):
                self._update(True)
        self._graph = (g1, g2)
        # the exchange form the graphs were captured around, fixed here: an eager step in between (test_step,
        # evaluate) rewrites self._overlapped with ITS form
        self._graph_overlapped = self._overlapped
        torch.cuda.synchronize(self.device)

    def _replay(self):
        g1, g2 = self._graph
        self._overlapped = self._graph_overlapped
        g1.replay()
        if g2 is not None:
            # split graphs: the whole bucket is exchanged between them (the per-level collectives are captured only
            # in the one-graph form)
            assert not self._graph_overlapped
            self._exchange()
            g2.replay()

    # ------------------------------------------------------------------ inference API
    def _level_forward_only(self, x, l, training):
        """vqvaes[l](x, training): forward of one level; with training the VQ EMA runs (VectorQuantizer.py:
        116-145) — under data parallelism on the statistics of the GLOBAL batch (this level's region of the
        bucket is all-reduced first), so the replicas' codebooks stay identical."""
        vq = self.vqs[l]
        with torch.no_grad():
            z = self.encoders[l].forward(x)
            if training:
                vq.stats.zero_()
                n_loc = z.shape[0] * z.shape[1]
                row_offset, n_global = vqa_dp.global_row_range(n_loc, self.process_group)
                q, _ = vq.forward(z, training=True, row_offset=row_offset, n_global=n_global)
                vqa_dp.exchange(vq.stats, self.process_group)
                vq.apply_ema()
            else:
                q, _ = vq.forward(z, training=False)
            return self.decoders[l].forward(q)

    def __call__(self, x, training=False):
        """vqvae.py:178-206 -> (recons, {level_losses, recon_losses, commit_losses, spec_losses})."""
        if isinstance(x, tuple):
            x = x[0]
        x = self._as_input(x)
        target = SpectralTarget(x)
        recons, out = [], {"level_losses": [], "recon_losses": [], "commit_losses": [], "spec_losses": []}
        with torch.no_grad():
            for l in range(self.levels):
                r = self._level_forward_only(x, l, training)
                recons.append(r)
                spec, _ = multispectral_loss_and_grad(target, r, need_grad=False)
                spec = spec[0]
                recon = ((x - r) ** 2).mean()
                commit = self.vqs[l].commit[0].clone()
                out["level_losses"].append(recon + commit + spec)
                out["recon_losses"].append(recon)
                out["commit_losses"].append(commit)
                out["spec_losses"].append(spec)
        return recons, out

    call = __call__

    def encode_level(self, x, level, chunk=1):
        """vqvae.py:208-219 -> (B, T_l) int64 codes."""
        x = self._as_input(x)
        with torch.no_grad():
            z = self.encoders[level].forward(x)
            idx = self.vqs[level].get_code_indices(z.reshape(-1, self.latent_dim))
        return idx.view(z.shape[0], z.shape[1])

    def encode(self, x, start_level=0, end_level=None):
        end_level = self.levels if end_level is None else end_level
        return [self.encode_level(x, l) for l in range(start_level, end_level)]

    def decode_level(self, zq, level, chunk=1):
        """vqvae.py:238-251: one_hot(zq) @ E^T (a row gather of ET) -> decoder."""
        zq = torch.as_tensor(zq, device=self.device).long()
        with torch.no_grad():
            q = self.vqs[level].ET[zq.reshape(-1)].view(*zq.shape, self.latent_dim).to(self.cdt).contiguous()
            return self.decoders[level].forward(q)

    def decode(self, zq, level=0):
        return self.decode_level(zq, level)

    # ------------------------------------------------------------------ training loop / state
    def fit(self, x=None, y=None, batch_size=32, epochs=1, shuffle=True, seed=0, verbose=0):
        """Minimal keras fit: `self.metrics` reset per epoch (keras semantics); returns the history of
        epoch-end results."""
        if self.optimizer is None:
            self.compile()
        xs = np.asarray(x, np.float32)
        n = xs.shape[0]
        rng = np.random.default_rng(seed)
        hist = []
        for ep in range(epochs):
            self.reset_metrics()
            order = rng.permutation(n) if shuffle else np.arange(n)
            for i in range(0, n - batch_size + 1, batch_size):
                self.train_step(xs[order[i:i + batch_size]])
            res = {k: float(v) for k, v in self.results().items()}
            hist.append(res)
            if verbose:
                print(f"epoch {ep + 1}/{epochs}", res)
        return hist

    def get_weights(self) -> Dict[str, np.ndarray]:
        return self.store.values()

    def set_weights(self, vals: Dict[str, np.ndarray]):
        self.store.set_values(vals)

    def get_vq_state(self):
        return [vq.get_state() for vq in self.vqs]

    def set_vq_state(self, states):
        for vq, st in zip(self.vqs, states):
            vq.set_state(st)

    @property
    def trainable_variables(self):
        return list(chain.from_iterable(m.trainable_variables for m in self.vqvaes))

    def state_dict(self):
        """Checkpoint payload: weights, Adam moments and step, VQ state."""
        sd = {"weights": self.store.flat.detach().cpu().clone(), "vq": self.get_vq_state()}
        if self.optimizer is not None and self.optimizer.m is not None:
            sd.update({"adam_m": self.optimizer.m.cpu().clone(), "adam_v": self.optimizer.v.cpu().clone(),
                       "iterations": int(self.optimizer.iterations.item())})
        return sd

    def save(self, path: str):
        """Checkpoint to disk (the reference saves through an injected tf.train.CheckpointManager every
        ckpt_interval epochs, src/callback/vae_monitor.py:56-58): tensors, ints and strings only, so
        `torch.load(path, weights_only=True)` reads it. Holds the weights, Adam moments and step, and each
        level's codebook E, m_t, N_t and reset counter: resuming reproduces the uninterrupted run bit for
        bit (every reduction of the step runs in a fixed order)."""
        sd = self.state_dict()
        out = {"format": f"vqa-vqvae/{CKPT_VERSION}", "param_names": [n for n, _, _ in self.store.specs],
               "layout": self.store.layout_record(),
               "config": {"input_shape": list(self.input_shape), "levels": self.levels,
                          "latent_dim": self.latent_dim, "num_embeddings": self.num_embeddings,
                          "down_depth": list(self.down_depth), "strides": list(self.strides)},
               "weights": sd["weights"]}
        for k in ("adam_m", "adam_v", "iterations"):
            if k in sd:
                out[k] = sd[k]
        for l, st in enumerate(sd["vq"]):
            for k in ("embeddings", "m_t", "N_t"):
                out[f"vq{l}/{k}"] = torch.from_numpy(np.ascontiguousarray(st[k]))
            out[f"vq{l}/calls"] = int(st["calls"])
        torch.save(out, path)

    def load(self, path: str):
        """Restore a `save` checkpoint (loaded weights-only: nothing in the file is executed). Format /2 records
        each tensor's offset, and the weights and Adam moments are copied tensor by tensor into this model's
        layout; a /1 file is read in the layout its length identifies (aligned or the earlier packed one)."""
        ck = torch.load(path, map_location="cpu", weights_only=True)
        lay = checkpoint_layout(ck, self.store, "vqvae", path)
        if ck.get("config", {}).get("levels", self.levels) != self.levels:
            raise ValueError(f"{path}: {ck['config']['levels']} levels, this model {self.levels}")
        sd = {"weights": self.store.from_layout(ck["weights"], lay, path),
              "vq": [{k: ck[f"vq{l}/{k}"].numpy() for k in ("embeddings", "m_t", "N_t")}
                     | {"calls": ck[f"vq{l}/calls"]} for l in range(self.levels)]}
        for k in ("adam_m", "adam_v"):
            if k in ck:
                sd[k] = self.store.from_layout(ck[k], lay, f"{path} ({k})")
        if "iterations" in ck:
            sd["iterations"] = ck["iterations"]
        self.load_state_dict(sd)

    def load_state_dict(self, sd):
        self.store.flat.copy_(sd["weights"].to(self.device))
        self.set_vq_state(sd["vq"])
        if "adam_m" in sd:
            if self.optimizer is None:
                self.compile()
            self.optimizer.m.copy_(sd["adam_m"].to(self.device))
            self.optimizer.v.copy_(sd["adam_v"].to(self.device))
            self.optimizer.iterations.fill_(int(sd["iterations"]))
