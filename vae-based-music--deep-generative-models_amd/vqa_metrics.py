"""keras.metrics.Mean equivalents kept on the device (no host sync per step; graph-capturable).

`Mean` owns its (total, count) pair. `SlotMean` is a tracker over one row of a model-owned accumulator
(the VQVAE keeps every tracker of a step in one (n, 2) tensor that a single libvqa launch updates,
vqa_step_metrics); both expose the Keras tracker surface the reference's callers use: `.name`,
`.update_state(v)`, `.result()`, `.reset_state()` (src/callback/vae_monitor.py:64-65,71).
"""
from __future__ import annotations

import torch


class Mean:
    def __init__(self, name: str, device):
        self.name = name
        self._acc = torch.zeros(2, dtype=torch.float32, device=device)  # [total, count]

    def update_state(self, value: torch.Tensor):
        self._acc[0].add_(value.reshape(()).to(torch.float32))
        self._acc[1].add_(1.0)

    def result(self) -> torch.Tensor:
        return self._acc[0] / self._acc[1].clamp(min=1.0)

    def reset_state(self):
        self._acc.zero_()

    # keras 2.x alias
    reset_states = reset_state


class SlotMean(Mean):
    """Mean over row `row` of a shared (n, 2) [total, count] accumulator."""

    def __init__(self, name: str, acc: torch.Tensor, row: int):
        self.name = name
        self._acc = acc[row]
