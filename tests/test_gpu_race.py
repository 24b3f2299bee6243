"""Cross-stream ordering of the train step under random delays (the `inject` experiment of tools/cotenant.py as a
test).

The step runs its levels' chains on concurrent HIP streams and joins them through events. A missing dependency
between streams would make the result depend on timing. Here, in one process, the step's local gradient (and its
EMA statistics and losses: the whole bucket) with the levels serialised on one stream is the reference; then the
step runs with the level streams overlapping while `vqa_lib.launch_hook` queues a random 10-400 µs spin on the
launching stream before ~15 % of the libvqa launches (every cross-stream order the step relies on is stretched both
ways). Every run must be BITWISE the serial one: the kernels are deterministic, so only an ordering bug can change
a bit.
"""
import os
import random
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import dp_worker as W  # noqa: E402
import vqa_lib  # noqa: E402

pytestmark = pytest.mark.gpu


def _bucket(config, dtype, B, serial, hook=None):
    old = W.B_LOCAL
    W.B_LOCAL = B
    try:
        m = W.build(B, config=config, dtype=dtype)
        x = m._as_input(W.batches(1, config)[0][:B])
    finally:
        W.B_LOCAL = old
    m.concurrent_levels = not serial
    torch.cuda.synchronize()
    vqa_lib.launch_hook = hook
    try:
        m._compute(x, True)
    finally:
        vqa_lib.launch_hook = None
    torch.cuda.synchronize()
    g = m.bucket.detach().cpu().clone()
    del m
    torch.cuda.empty_cache()
    return g


def _delay_hook(rng, p):
    def hook():
        if rng.random() < p:
            torch.cuda._sleep(rng.randint(25_000, 1_000_000))  # ~10-400 us at the shader clock
    return hook


@pytest.mark.timeout(600)
def test_concurrent_levels_with_random_delays_bitwise_equal_serial(cuda):
    config, dtype, B = "cfg2_short", "bf16", 2
    ref = _bucket(config, dtype, B, serial=True)
    bad = []
    for i in range(4):
        g = _bucket(config, dtype, B, serial=False, hook=_delay_hook(random.Random(1000 + i), 0.15))
        n = int((g != ref).sum())
        if n:
            bad.append(f"delay pattern {i}: {n} of {g.numel()} bucket elements differ")
    g = _bucket(config, dtype, B, serial=False)
    n = int((g != ref).sum())
    if n:
        bad.append(f"no delays: {n} differ")
    assert not bad, bad
