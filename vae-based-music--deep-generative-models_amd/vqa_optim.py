"""keras.optimizers.Adam (TF 2.7 defaults) over a ParamStore: one libvqa launch per step.

Keras' Adam hands each variable to TF's ApplyAdam with lr_t = lr*sqrt(1-b2^t)/(1-b1^t) and eps = 1e-7
applied after the bias correction (not PyTorch's form). `iterations` lives on the device so a captured
train step replays with the right t. `learning_rate` is a float or a keras LearningRateSchedule
(schedules.CustomSchedule — src/transformer/multi_head_attention.py:82-101 — or ExponentialDecay): a schedule
is evaluated on the device from `iterations` (vqa_lr_schedule) right before the update, so graph replay stays
valid.
"""
from __future__ import annotations

import torch

import vqa_lib as V
from schedules import LearningRateSchedule


class Adam:
    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7, **kwargs):
        if callable(learning_rate) and not isinstance(learning_rate, LearningRateSchedule):
            # a host callable cannot be evaluated inside a replayed hipGraph
            raise TypeError("learning_rate: a float or a schedules.LearningRateSchedule (device-evaluated)")
        self.learning_rate, self.beta_1, self.beta_2, self.epsilon = learning_rate, beta_1, beta_2, epsilon
        self.iterations = None
        self.m = self.v = None
        self._lr_dev = None

    @property
    def scheduled(self) -> bool:
        return isinstance(self.learning_rate, LearningRateSchedule)

    def build(self, store):
        dev = store.flat.device
        self.m = torch.zeros_like(store.flat)
        self.v = torch.zeros_like(store.flat)
        self.iterations = torch.zeros(1, dtype=torch.int64, device=dev)
        self._lr_dev = torch.zeros(1, dtype=torch.float32, device=dev) if self.scheduled else None

    def current_learning_rate(self) -> float:
        """The rate the next apply() uses (host evaluation of the schedule at the device step count)."""
        if not self.scheduled:
            return float(self.learning_rate)
        return self.learning_rate(int(self.iterations.item()))

    def apply(self, store, grad_scale: float = 1.0):
        if self.m is None:
            self.build(store)
        lr = 0.0
        if self.scheduled:
            kind, p = self.learning_rate.device_spec()
            V.lr_schedule(self.iterations, self._lr_dev, kind, p)
        else:
            lr = self.learning_rate
        V.adam_keras(store.flat, store.grad[:store.size], self.m, self.v, self.iterations, lr,
                     self.beta_1, self.beta_2, self.epsilon, grad_scale, lr_dev=self._lr_dev)
        V.counter_add(self.iterations, 1)
