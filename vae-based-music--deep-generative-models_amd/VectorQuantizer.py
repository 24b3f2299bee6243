"""EMA vector quantizer — drop-in for the reference VectorQuantizer.py (VectorQuantizer class).

State (VectorQuantizer.py:38-60): embeddings E (D, K) non-trainable, m_t (D, K) = E, N_t (K,) = 1.
call(x, training=True) (:75-165): nearest code (get_code_indices :170-186), q = E[:, idx],
commitment loss beta * mean((sg(q) - x)^2) (:97-107), straight-through x + sg(q - x) (:114), and when
training the EMA update with dead-code reset (:116-145) and usage / entropy metrics (:149-159).

MI355X path: libvqa kernels — an MFMA argmin that never materialises the N x K distances (bf16 MFMA on
exact hi/mid/lo planes of E when z is bf16), a row gather
from ET = E^T (the one-hot GEMM of :86-90 is a gather), atomic EMA sums (the dense GEMM of :123-124 is
a scatter-add), and one EMA/reset kernel. The reset candidates use an injected seeded permutation in
place of the reference's unseeded tf.random.shuffle (:137).

Inside VQVAE.train_step the EMA statistics are written into the model's all-reduce bucket during the
forward and applied after the (data-parallel) exchange — numerically the same as the reference, which
updates E after quantising and never reuses the new E within the step.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

import vqa_lib as V
from vqa_metrics import Mean, SlotMean


class VectorQuantizer:
    def __init__(self, num_embeddings, embedding_dim, beta=0.25, codebook_usage_threshold=1.0, decay_rate=0.99,
                 level=0, name=None, *, device="cuda", seed=2, reset_seed=3, **kwargs):
        self.num_embeddings, self.embedding_dim = num_embeddings, embedding_dim
        self.beta = beta
        self.codebook_usage_threshold = codebook_usage_threshold
        self.gamma = decay_rate
        self.level = level
        self.name = name or f"vector_quantizer_{level}"
        self.reset_seed = reset_seed
        self.device = torch.device(device)
        D, K = embedding_dim, num_embeddings
        rng = np.random.default_rng(seed)
        E = rng.uniform(-0.05, 0.05, size=(D, K)).astype(np.float32)  # tf.random_uniform_initializer()
        self.embeddings = torch.from_numpy(E).to(self.device)
        self.ET = self.embeddings.t().contiguous()
        self.m_t = self.embeddings.clone()
        self.N_t = torch.ones(K, dtype=torch.float32, device=self.device)
        self.e_sqnorm = torch.empty(K, dtype=torch.float32, device=self.device)
        # hi/mid/lo bf16 planes of E for the bf16-MFMA argmin (exact products; vqa_vq_argmin_split)
        self.E3 = torch.empty(K, 3, D, dtype=torch.bfloat16, device=self.device)
        self.calls = torch.zeros(1, dtype=torch.int64, device=self.device)  # reset-permutation counter
        self.vq_metrics = torch.zeros(3, dtype=torch.float32, device=self.device)
        self.commit = torch.zeros(1, dtype=torch.float32, device=self.device)
        # EMA statistics: own buffers unless a model binds them into its all-reduce bucket
        self.bind_stats(torch.zeros(self.stats_size(), dtype=torch.float32, device=self.device))
        self._codebook_changed()
        # TF multiplies float32 tensors by the python floats gamma and (1. - gamma) (:128,:131)
        self._g = float(np.float32(decay_rate))
        self._omg = float(np.float32(1.0 - decay_rate))
        self.batch_usage_tracker = Mean(f"[{level}]batch_codebook_usage", self.device)
        self.usage_tracker = Mean(f"[{level}]codebook_usage", self.device)
        self.entropy_tracker = Mean(f"[{level}]codebook_entropy", self.device)
        self._saved = None

    @property
    def metrics(self):
        return [self.batch_usage_tracker, self.usage_tracker, self.entropy_tracker]

    def bind_metrics(self, vq_metrics: torch.Tensor, macc: torch.Tensor, rows):
        """Inside a VQVAE: the per-step usage / entropy values live in the model's (levels, 3) buffer and the
        trackers are rows of its accumulator (updated by the model's one-launch vqa_step_metrics)."""
        self.vq_metrics = vq_metrics
        names = [m.name for m in self.metrics]
        self.batch_usage_tracker, self.usage_tracker, self.entropy_tracker = (
            SlotMean(n, macc, r) for n, r in zip(names, rows))

    # ---- statistics buffers (m_sumT (K, D) | n_sum (K) | RT (K, D)) ----
    def stats_size(self) -> int:
        K, D = self.num_embeddings, self.embedding_dim
        return 2 * K * D + K

    def bind_stats(self, buf: torch.Tensor):
        K, D = self.num_embeddings, self.embedding_dim
        assert buf.numel() == self.stats_size()
        self.stats = buf
        self.m_sumT = buf[:K * D].view(K, D)
        self.n_sum = buf[K * D:K * D + K]
        self.RT = buf[K * D + K:].view(K, D)

    def _codebook_changed(self):
        """Derived codebook state after every change of E: |e_k|^2 and the bf16 planes."""
        V.vq_sqnorm(self.embeddings, self.e_sqnorm)
        V.vq_split_bf16x3(self.embeddings, self.E3)

    def _argmin(self, flat: torch.Tensor, idx: torch.Tensor, min_dist=None):
        if flat.dtype == torch.bfloat16 and self.embedding_dim in (32, 64):
            V.vq_argmin_split(flat, self.E3, self.e_sqnorm, idx, min_dist)
        else:
            V.vq_argmin(flat, self.embeddings, self.e_sqnorm, idx, min_dist)

    # ---- reference API ----
    def get_code_indices(self, flattened_inputs: torch.Tensor) -> torch.Tensor:
        """VectorQuantizer.py:170-186 -> (N,) int64, ties to the lowest index."""
        flat = flattened_inputs.contiguous()
        idx = torch.empty(flat.shape[0], dtype=torch.int64, device=flat.device)
        self._argmin(flat, idx)
        return idx

    def _tile(self, x):
        """VectorQuantizer.py:191-199: rows repeated ceil(K / N) times when N < K (so K candidate rows exist for
        the dead-code reset). The product's reset draws the same rows by index (vqa_reset_perm_index takes the
        row modulo N) without forming this tensor; this is the host-side form of the reference helper."""
        x = torch.as_tensor(x)
        nt, k = x.shape[0], self.num_embeddings
        if nt < k:
            return x.repeat((k + nt - 1) // nt, *([1] * (x.dim() - 1)))
        return x

    def get_usage_count(self):
        return self.N_t

    def call(self, x, training=True, debug=False):
        """Standalone use (VectorQuantizer.py:75-165): the EMA update is applied immediately."""
        self.stats.zero_()
        q, idx = self.forward(x, training=training, row_offset=0, n_global=None)
        if training:
            self.apply_ema()
        if debug:
            print("VQ input (Encoder Output): ", x)
            print("VQ output: ", q)
        return q, idx

    __call__ = call

    @property
    def losses(self):
        return [self.commit[0]]

    # ---- split forward / EMA for the train step ----
    def forward(self, z: torch.Tensor, training: bool, row_offset: int = 0, n_global: Optional[int] = None,
                save: bool = False):
        """Quantise z (B, T, D). Writes the commitment loss to self.commit; when training, accumulates the
        EMA sums into the bound stats buffer (caller zeroes it) and the reset candidates into RT."""
        D = self.embedding_dim
        flat = z.reshape(-1, D)
        N = flat.shape[0]
        idx = torch.empty(N, dtype=torch.int64, device=z.device)
        self._argmin(flat, idx)
        q = torch.empty_like(flat)
        V.vq_quantize(flat, self.ET, idx, q, self.commit, self.m_sumT if training else None,
                      self.n_sum if training else None, self.beta)
        if training:
            V.vq_reset_rows(flat, self.RT, row_offset, n_global or N, self.reset_seed, self.calls, self.level)
        self._saved = (flat, idx) if save else None
        return q.view(z.shape), idx

    def backward(self, dq: torch.Tensor, n_global: Optional[int] = None):
        """dz = dq (straight-through) + 2*beta*(z - q)/(N_global*D) (commitment gradient)."""
        flat, idx = self._saved
        self._saved = None
        D = self.embedding_dim
        n = n_global or flat.shape[0]
        dz = torch.empty_like(flat)
        V.vq_backward(dq.reshape(-1, D), flat, self.ET, idx, dz, float(2.0 * self.beta / (n * D)))
        return dz.view(dq.shape)

    def apply_ema(self, update_trackers: bool = True):
        # the new codebook's |e|^2 and bf16 planes (the next argmin's inputs) come out of the same launch
        V.vq_ema_apply(self.embeddings, self.ET, self.m_t, self.N_t, self.m_sumT, self.n_sum, self.RT, self._g,
                       self._omg, float(self.codebook_usage_threshold), self.vq_metrics, self.calls,
                       esq=self.e_sqnorm, E3=self.E3)
        if update_trackers:
            self.batch_usage_tracker.update_state(self.vq_metrics[0])
            self.usage_tracker.update_state(self.vq_metrics[1])
            self.entropy_tracker.update_state(self.vq_metrics[2])

    # ---- state ----
    def get_state(self):
        return {"embeddings": self.embeddings.cpu().numpy().copy(), "m_t": self.m_t.cpu().numpy().copy(),
                "N_t": self.N_t.cpu().numpy().copy(), "calls": int(self.calls.item())}

    def set_state(self, st):
        self.embeddings.copy_(torch.as_tensor(np.asarray(st["embeddings"], np.float32)))
        self.ET.copy_(self.embeddings.t())
        self.m_t.copy_(torch.as_tensor(np.asarray(st["m_t"], np.float32)))
        self.N_t.copy_(torch.as_tensor(np.asarray(st["N_t"], np.float32)))
        self.calls.fill_(int(st.get("calls", 0)))
        self._codebook_changed()
