"""Injected dead-code-reset permutation — numpy restatement (integer-exact). TEST INFRASTRUCTURE ONLY.

The reference draws reset candidates with an UNSEEDED `tf.random.shuffle(self._tile(flattened))[:K]`
(VectorQuantizer.py:137, _tile :191-199). A parity build must inject the permutation; ours is a keyed
4-round balanced Feistel bijection on [0, 2^(2h)) cycle-walked into [0, M) (M = tiled row count), keyed
by (seed, per-quantizer call counter, level). This file restates it bit-for-bit from its definition so
tests can check the product's implementation (vqa_common.h perm_index / vqa_reset_perm_index).
"""
import numpy as np

_M64 = (1 << 64) - 1
_M32 = (1 << 32) - 1


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def perm_key(seed: int, counter: int, level: int) -> int:
    return splitmix64((splitmix64((seed + level) & _M64) + counter) & _M64)


def _mix32(x):
    x = np.asarray(x, dtype=np.uint64) & _M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & np.uint64(_M32)
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & np.uint64(_M32)
    x ^= x >> np.uint64(16)
    return x


def perm_indices(key: int, M: int, ks) -> np.ndarray:
    """perm(k) for every k in ks (vectorised), a bijection of [0, M)."""
    h = 1
    while (1 << (2 * h)) < M:
        h += 1
    mask = np.uint64((1 << h) - 1)
    k0, k1 = key & _M32, (key >> 32) & _M32
    rk = [k0, k1, k0 ^ 0x9E3779B9, k1 ^ 0x85EBCA6B]
    x = np.asarray(ks, dtype=np.uint64).copy()
    todo = np.ones(x.shape, dtype=bool)
    while todo.any():
        xs = x[todo]
        L = (xs >> np.uint64(h)) & mask
        R = xs & mask
        for r in range(4):
            F = _mix32(((R ^ np.uint64(rk[r])) + np.uint64(r)) & np.uint64(_M32)) & mask
            L, R = R, L ^ F
        xs = (L << np.uint64(h)) | R
        x[todo] = xs
        todo[todo] = xs >= np.uint64(M)
    return x.astype(np.int64)


def reset_rows(seed: int, counter: int, level: int, n_rows: int, K: int) -> np.ndarray:
    """Row indices (into the un-tiled batch of n_rows) that `shuffle(tile(flat))[:K]` selects."""
    M = n_rows if n_rows >= K else n_rows * ((K + n_rows - 1) // n_rows)
    return perm_indices(perm_key(seed, counter, level), M, np.arange(K)) % n_rows
