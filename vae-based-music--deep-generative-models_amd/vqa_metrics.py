"""keras.metrics.Mean equivalent kept on the device (no host sync per step; graph-capturable)."""
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
