"""VQVAESampler — drop-in for the reference's Sampler.py:10-136 (BASELINE config 5's ancestral decode).

Top-down sampling over the VQ-VAE's levels: the top prior samples one window of codes; every lower prior (an
upsampler, conditioned through its ConditionerNet on the level above) samples its window conditioned on the codes
just drawn above it. Each window is ONE persistent decode launch (Prior.sample -> vqa_prior_decode): the KV-cache
kernel walks the positions on the device, so the whole multi-level draw is `levels` launches plus the
conditioners' up-sampling — no per-token host round trip and no per-token graph replay.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from prior import Prior


class VQVAESampler:
    """Sampler.py:10-63. n_ctxs[l]: the context (window) length of level l's prior, in that level's codes."""

    def __init__(self, down_depth, strides, n_ctxs, codebook_size=513, priors: Optional[List[Prior]] = None,
                 num_genres=None, dtype="fp32", device="cuda", seed=1, **kwargs):
        self.downsamples = [stride ** down for stride, down in zip(strides, down_depth)]
        self.hop_lengths = np.cumprod(self.downsamples)
        self.levels = len(down_depth)
        self.bins = codebook_size
        # Sampler.py:24-25
        self.x_cond_kwargs = dict(dilation_factor=3, dilation_cycle=4, residual_width=32, residual_depth=8)
        self.prior_kwargs = dict(width=128, depth=6, heads=2, blocks=4, attn_stacks=1, drop_out_rate=0.0)
        self.priors: List[Prior] = []
        if priors is not None:
            assert len(priors) == self.levels
            self.priors = list(priors)
            return

        def rescale(level, cur_level):  # Sampler.py:21-22
            return (n_ctxs[cur_level] * int(self.hop_lengths[cur_level]) // int(self.hop_lengths[level]),)

        for l in range(self.levels):
            zs_shapes = [rescale(l_, l) for l_ in range(self.levels)]
            assert zs_shapes[l][0] == n_ctxs[l]
            x_cond_kwargs = self.x_cond_kwargs if l != self.levels - 1 else None
            self.priors.append(Prior(level=l, z_shapes=zs_shapes, bins=self.bins, down_depth=down_depth,
                                     strides=strides, vqvae_model=None, prior_kwargs=self.prior_kwargs,
                                     x_cond_kwargs=x_cond_kwargs, genre_classes=num_genres, dtype=dtype,
                                     device=device, seed=seed + l))

    def sample(self, n_samples, y_genre=None, seed=0):
        """Sampler.py:65-114: from the top level down; returns [zs_0, ..., zs_{L-1}], (n_samples, n_ctx_l) int64
        codes without the start token. Level l draws its Gumbel noise with seed + l."""
        dev = self.priors[0].device
        zs = [torch.zeros(n_samples, 0, dtype=torch.int64, device=dev) for _ in range(self.levels)]
        for level in reversed(range(self.levels)):
            pr = self.priors[level]
            x_cond = pr.get_cond(zs, 0, pr.context_length)
            seq = pr.sample(n_samples=n_samples, z_cond=x_cond, y=y_genre, seed=seed + level)
            zs[level] = torch.cat([zs[level], seq[:, 1:]], dim=-1)  # the start token removed (Sampler.py:108)
        return zs

    def sample_level(self, zs, level):
        """Sampler.py:116-124 (a stub in the reference)."""
        return NotImplementedError
