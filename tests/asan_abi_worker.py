"""Host-side AddressSanitizer pass over the C-ABI (tests/test_asan_abi.py; not collected by pytest).

Loads the ASan build (`make -C csrc asan` -> build_asan/libvqa_asan.so: -fsanitize=address on the host
compilation only) without a GPU and drives every host path that needs none:
  - every status-returning entry point with NULL device pointers (and a few size patterns) must be REJECTED by
    its argument validation (non-zero status, an error text) — never dereference a NULL host array, never
    reach a launch, never divide by a zero stride;
  - the workspace / support / padding queries over the model's shapes and edge shapes;
  - `vqa_reduce_partials` over a host descriptor array (its loop reads exactly `count` descriptors);
  - `vqa_reset_perm_index` over a range.
Any heap / stack / global overflow or use-after-free in that host code aborts the process with an ASan report.
    LD_PRELOAD=<libclang_rt.asan-x86_64.so> python tests/asan_abi_worker.py LIB path/to/vqa_lib.py
"""
import ctypes
import sys

LIB = sys.argv[1]
L = ctypes.CDLL(LIB)

P, I, L64, S, F, U = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t, ctypes.c_float, ctypes.c_uint64

# the ctypes table of the product binding, read from its source (vqa_lib imports torch, which this ASan process
# does not load): the `_SIGS = {...}` literal evaluates with the aliases above
src = open(sys.argv[2]).read()
start = src.index("_SIGS = {")
end = src.index("\n}\n", start) + 2
ns = {"ctypes": ctypes, "_P": P, "_I": I, "_L": L64, "_S": S, "_F": F, "_U": U,
      "_CONV": [I] * 11, "_CONVT": [I] * 10}
exec(src[start:end], ns)  # noqa: S102 — the repository's own binding table
SIGS = ns["_SIGS"]

L.vqa_get_last_error.restype = ctypes.c_char_p
for name, (res, args) in SIGS.items():
    fn = getattr(L, name)
    fn.restype = res
    fn.argtypes = args


def value(t, k):
    if t is P:
        return None
    if t in (I, L64):
        return (1, 0, -1, 64, 1 << 20)[k]
    if t in (S, U):
        return (0, 16, 1 << 40, 0, 1)[k]
    return (0.0, 1.0, -1.0, 0.5, 1e30)[k]


n_rejected = 0
accepted = []
for name, (res, args) in SIGS.items():
    if res is not I or P not in args:
        continue
    for k in range(5):
        rc = getattr(L, name)(*[value(t, k) for t in args])
        if rc == 0:
            accepted.append((name, k))
        else:
            n_rejected += 1
            assert L.vqa_get_last_error(), f"{name}: status {rc} without an error text"
# size / support queries: any integer pattern returns a value (0 or -1 for an unsupported shape), never traps
for name, (res, args) in SIGS.items():
    if res in (S, L64) and P not in args and name.endswith("workspace"):
        for k in range(5):
            getattr(L, name)(*[value(t, k) for t in args])
for k in range(5):
    L.vqa_same_out_len(value(I, k), value(I, (k + 1) % 5) - 1)
    L.vqa_same_pad_left(value(I, k), value(I, (k + 2) % 5), value(I, (k + 1) % 5) - 1, value(I, k) - 1)
# a status entry point may accept NULL pointers only where a NULL is an optional input with nothing to do
# (no GPU here: a call that got as far as a launch would fail and report a status, but none may get there)
bad = [a for a in accepted if a[0] not in ("vqa_reduce_partials",)]
assert not bad, f"entry points that accepted NULL device pointers: {bad}"

# queries over the model's shapes and edge shapes
for B, T in ((1, 1), (2, 7), (32, 65536), (32, 32768), (8, 8192)):
    for C, O, K, st, dil in ((1, 32, 3, 2, 1), (32, 32, 3, 1, 9), (32, 64, 3, 1, 1), (64, 32, 4, 2, 1)):
        To = L.vqa_same_out_len(T, st)
        pad = L.vqa_same_pad_left(T, K, st, dil)
        assert To >= 1 and pad >= 0
        for dt in (0, 1):
            L.vqa_conv1d_bwd_weight_workspace(B, T, To, C, O, K, st, dil, pad, 0, dt)
            L.vqa_conv1d_bwd_data_weight_workspace(B, T, To, C, O, K, st, dil, pad, 0, dt)
            L.vqa_conv1d_transpose_bwd_weight_workspace(B, T, T * st, C, O, K, st, 0, 0, dt)
    for d in (1, 3, 9, 27, 0, 1 << 20):
        for dt in (0, 1, 7):
            L.vqa_resblock_supported(32, d, dt)
            L.vqa_resblock_supported(31, d, dt)

# reduce_partials reads exactly `count` host descriptors (more than one batch of them here)
class Desc(ctypes.Structure):
    _fields_ = [("partials", P), ("dw", P), ("db", P), ("nparts", I), ("n", I), ("n_w", I), ("reserved", I)]


for count in (1, 7, 33, 100):
    arr = (Desc * count)()
    assert L.vqa_reduce_partials(arr, count, None) != 0  # NULL partials: rejected
assert L.vqa_reduce_partials(None, 3, None) != 0
assert L.vqa_reduce_partials(None, 0, None) == 0  # nothing to reduce

for M in (1, 2, 4096, 1 << 20):
    for k in sorted({0, M // 2, M - 1}):
        for lvl in (0, 2):
            v = L.vqa_reset_perm_index(7, 3, lvl, M, k)
            assert 0 <= v < M, (M, k, v)
    assert L.vqa_reset_perm_index(7, 3, 0, M, M) < 0 and L.vqa_reset_perm_index(7, 3, 0, M, -1) < 0
assert sorted(L.vqa_reset_perm_index(7, 3, 1, 1000, k) for k in range(1000)) == list(range(1000))  # a permutation

print(f"asan host pass ok: {n_rejected} NULL-pointer calls rejected, accepted {accepted}")
