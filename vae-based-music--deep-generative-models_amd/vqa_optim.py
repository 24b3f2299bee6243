"""keras.optimizers.Adam (TF 2.7 defaults) over a ParamStore: one libvqa launch per step.

Keras' Adam hands each variable to TF's ApplyAdam with lr_t = lr*sqrt(1-b2^t)/(1-b1^t) and eps = 1e-7
applied after the bias correction (not PyTorch's form). `iterations` lives on the device so a captured
train step replays with the right t.
"""
from __future__ import annotations

import torch

import vqa_lib as V


class Adam:
    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7, **kwargs):
        self.learning_rate, self.beta_1, self.beta_2, self.epsilon = learning_rate, beta_1, beta_2, epsilon
        self.iterations = None
        self.m = self.v = None

    def build(self, store):
        dev = store.flat.device
        self.m = torch.zeros_like(store.flat)
        self.v = torch.zeros_like(store.flat)
        self.iterations = torch.zeros(1, dtype=torch.int64, device=dev)

    def apply(self, store, grad_scale: float = 1.0):
        if self.m is None:
            self.build(store)
        V.adam_keras(store.flat, store.grad[:store.size], self.m, self.v, self.iterations, self.learning_rate,
                     self.beta_1, self.beta_2, self.epsilon, grad_scale)
        V.counter_add(self.iterations, 1)
