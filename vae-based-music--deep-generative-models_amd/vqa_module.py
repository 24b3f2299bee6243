"""Keras-like layer base: deferred build, standalone __call__, explicit forward/backward.

A layer registers its weights in a ParamStore at build() (the input channel count is known then, as
in Keras' deferred build). Used standalone, `layer(x)` builds a private store on first call with the
Keras default initialisers and runs the forward on the GPU. Inside VQVAE every layer shares the model's
store so the whole model's weights / gradients are two flat buffers.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from vqa_layers import ParamStore


class Layer:
    def __init__(self, name: Optional[str] = None, **kwargs):
        self.name = name or type(self).__name__
        self.built = False
        self.cdt = torch.float32
        self.store: Optional[ParamStore] = None

    # subclasses implement _build(store, prefix, input_dim) -> output_dim, forward, backward
    def build(self, store: ParamStore, prefix: str, input_dim: int, cdt: torch.dtype) -> int:
        self.store, self.cdt = store, cdt
        out = self._build(store, prefix, input_dim)
        self.built = True
        return out

    def _standalone_build(self, x: torch.Tensor, seed: int = 1):
        store = ParamStore()
        cdt = x.dtype if x.dtype in (torch.float32, torch.bfloat16) else torch.float32
        self.build(store, self.name, x.shape[-1], cdt)
        store.materialize(x.device, seed=seed)

    def __call__(self, x: torch.Tensor, training: bool = False, **kwargs) -> torch.Tensor:
        if not self.built:
            self._standalone_build(x)
        return self.forward(x, save=False)

    def forward(self, x, save=False):
        raise NotImplementedError

    def backward(self, dy):
        raise NotImplementedError

    @property
    def weights(self):
        return {n: self.store.view(n) for n in self._param_names()} if self.store else {}

    def _param_names(self):
        return []


def _is_array(a) -> bool:
    return isinstance(a, (torch.Tensor, np.ndarray))


def keras_evaluate(model, x=None, y=None, batch_size=None, verbose=0, steps=None, return_dict=False):
    """keras Model.evaluate (TF 2.7 semantics) over `model.test_step`, as the reference's monitors call it
    (src/callback/vae_monitor.py:69, src/callback/monitors.py:81: `self.model.evaluate(self.val_dataset)`):
      - the model's metrics are reset first (`model.reset_metrics()`), then `test_step` runs on every batch —
        for the VQ-VAE that includes the codebook EMA update (VectorQuantizer.py:75 defaults training=True);
      - `x` is a dataset-like iterable of batches (each a tensor / array or a tuple (x, y, ...), as tf.data
        yields them), or an array (optionally with `y`) cut into `batch_size` rows (default 32, the last batch
        partial); `steps` caps the number of batches;
      - returns the last step's logs (the trackers' running means) as a dict of floats with `return_dict`,
        otherwise keras' flatten_metrics_in_order: the values whose keys are tracker names first, in
        `model.metrics` order, then the other keys sorted; a single value is returned bare."""
    if x is None:
        raise ValueError("evaluate needs data")
    if isinstance(x, tuple) and len(x) == 2 and _is_array(x[0]) and y is None:
        x, y = x
    if _is_array(x):
        n = int(x.shape[0])
        bs = int(batch_size or 32)
        if y is not None and int(y.shape[0]) != n:
            raise ValueError(f"x has {n} rows, y {int(y.shape[0])}")
        batches = ((x[i:i + bs], y[i:i + bs]) if y is not None else x[i:i + bs] for i in range(0, n, bs))
    else:
        if y is not None:
            raise ValueError("`y` is only accepted with array inputs (a dataset yields (x, y) batches itself)")
        batches = iter(x)
    model.reset_metrics()
    logs = None
    for i, batch in enumerate(batches):
        if steps is not None and i >= steps:
            break
        logs = model.test_step(batch)
        if verbose:
            print(f"evaluate batch {i + 1}", {k: round(float(v), 6) for k, v in logs.items()})
    if logs is None:
        raise ValueError("evaluate got no batches")
    logs = {k: float(v) for k, v in logs.items()}
    if return_dict:
        return logs
    names = [m.name for m in model.metrics]
    out = [logs[k] for k in names if k in logs] + [logs[k] for k in sorted(logs) if k not in names]
    return out[0] if len(out) == 1 else out
