"""keras.optimizers.schedules for the product's Keras Adam (vqa_optim.Adam), evaluated ON THE DEVICE.

The reference's transformer schedule `CustomSchedule(d_model, warmup_steps=4000)`
(src/transformer/multi_head_attention.py:82-101) — lr(step) = rsqrt(d_model) * min(rsqrt(step), step *
warmup_steps^-1.5) — and keras' ExponentialDecay. Keras' OptimizerV2._decayed_lr calls the schedule with
float(iterations), the step count BEFORE the update's increment (so CustomSchedule gives 0 on the first step).

Each schedule is a Python callable with the reference's signature (host float32 value, for logging / tests)
and a `device_spec()` (kind, params) that vqa_lr_schedule evaluates from the optimizer's device step counter:
a captured train step therefore replays with the rate of the step it is replaying. The constants are rounded
to float32 on the host the way TF forms them (rsqrt of the float32 d_model; the Python-float power of the
integer warmup_steps cast to float32 by the multiply).
"""
from __future__ import annotations

import math

import numpy as np


class LearningRateSchedule:
    """keras.optimizers.schedules.LearningRateSchedule: subclasses give __call__(step) and device_spec()."""

    def __call__(self, step):
        raise NotImplementedError

    def device_spec(self):
        raise NotImplementedError

    def get_config(self):
        return {}


class CustomSchedule(LearningRateSchedule):
    """src/transformer/multi_head_attention.py:82-101 (the transformer warm-up / inverse-square-root schedule)."""

    def __init__(self, d_model, warmup_steps=4000):
        self.d_model = np.float32(d_model)  # tf.cast(d_model, tf.float32)
        self.warmup_steps = warmup_steps

    def _consts(self):
        rs_d = np.float32(1.0) / np.sqrt(self.d_model, dtype=np.float32)  # tf.math.rsqrt(d_model)
        w = np.float32(self.warmup_steps ** -1.5)  # python float, cast to float32 when it scales the step
        return rs_d, w

    def __call__(self, step):
        s = np.float32(step)
        rs_d, w = self._consts()
        with np.errstate(divide="ignore"):
            arg1 = np.float32(1.0) / np.sqrt(s, dtype=np.float32)  # tf.math.rsqrt(step): inf at step 0
        arg2 = np.float32(s * w)
        return float(np.float32(rs_d * np.minimum(arg1, arg2)))

    def device_spec(self):
        rs_d, w = self._consts()
        return 1, (float(rs_d), float(w))

    def get_config(self):
        return {"d_model": float(self.d_model), "warmup_steps": self.warmup_steps}


class ExponentialDecay(LearningRateSchedule):
    """keras.optimizers.schedules.ExponentialDecay: initial * decay_rate ** (step / decay_steps), the exponent
    floored when staircase."""

    def __init__(self, initial_learning_rate, decay_steps, decay_rate, staircase=False, name=None):
        if decay_steps <= 0:
            raise ValueError("decay_steps must be positive")
        self.initial_learning_rate, self.decay_steps = initial_learning_rate, decay_steps
        self.decay_rate, self.staircase = decay_rate, staircase

    def __call__(self, step):
        p = np.float32(np.float32(step) / np.float32(self.decay_steps))
        if self.staircase:
            p = np.float32(math.floor(p))
        return float(np.float32(np.float32(self.initial_learning_rate) *
                                np.float32(np.power(np.float32(self.decay_rate), p, dtype=np.float32))))

    def device_spec(self):
        return 2, (float(np.float32(self.initial_learning_rate)), float(np.float32(self.decay_steps)),
                   float(np.float32(self.decay_rate)), 1.0 if self.staircase else 0.0)

    def get_config(self):
        return {"initial_learning_rate": self.initial_learning_rate, "decay_steps": self.decay_steps,
                "decay_rate": self.decay_rate, "staircase": self.staircase}
