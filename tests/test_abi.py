"""C-ABI checks that need no GPU: libvqa.so loads, exports every symbol include/vqa.h declares, and its
host-callable functions agree with the oracle (TF SAME padding, the injected reset permutation)."""
import os
import re

import numpy as np
import pytest

import vqa_lib as V
from oracle import reset_perm
from oracle.vqvae_ref import same_pad

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "vqa.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(vqa_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    lib = V.lib()
    declared = _declared()
    assert len(declared) >= 20
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(V.EXPORTED) == declared


def test_version_and_error_string():
    assert b"gfx950" in V.lib().vqa_version()
    assert isinstance(V.last_error(), str)


def test_abi_revision_matches_header_and_binding():
    """include/vqa.h VQA_ABI_VERSION = the library's vqa_abi_version() = the binding's ABI_VERSION; a library of
    another revision is refused at load (a changed argument list would otherwise shift arguments silently)."""
    import re
    hdr = open(HEADER).read()
    want = int(re.search(r"#define VQA_ABI_VERSION (\d+)", hdr).group(1))
    assert V.lib().vqa_abi_version() == want == V.ABI_VERSION


@pytest.mark.parametrize("T,K,s,d", [(4096, 4, 2, 1), (4097, 4, 2, 1), (512, 3, 1, 27), (40, 3, 1, 27),
                                     (1000, 3, 1, 9), (7, 4, 2, 1), (65536, 3, 1, 1), (1, 3, 1, 1)])
def test_same_padding_matches_oracle(T, K, s, d):
    out, left, _ = same_pad(T, K, s, d)
    assert V.same_out_len(T, s) == out
    assert V.same_pad_left(T, K, s, d) == left


@pytest.mark.parametrize("M,level,counter", [(262144, 0, 0), (65536, 1, 7), (1024, 2, 3), (3000, 0, 1),
                                             (5, 0, 0), (2048, 1, 123456)])
def test_reset_permutation_host_matches_numpy(M, level, counter):
    ks = np.arange(min(M, 300))
    want = reset_perm.perm_indices(reset_perm.perm_key(3, counter, level), M, ks)
    got = np.array([V.reset_perm_index(3, counter, level, M, int(k)) for k in ks])
    assert np.array_equal(got, want)


def test_reset_permutation_is_a_bijection():
    for M in (5, 64, 1000, 4096):
        p = reset_perm.perm_indices(reset_perm.perm_key(3, 0, 0), M, np.arange(M))
        assert np.array_equal(np.sort(p), np.arange(M))


def test_reset_rows_tile_semantics():
    # N < K: rows are drawn from the tiled batch (VectorQuantizer._tile :191-199) -> every row index < N
    rows = reset_perm.reset_rows(3, 0, 0, 100, 1024)
    assert rows.shape == (1024,) and rows.max() < 100 and rows.min() >= 0
    # N >= K: K distinct rows
    rows = reset_perm.reset_rows(3, 0, 0, 5000, 2048)
    assert len(np.unique(rows)) == 2048


def test_decoder_tail_rejects_more_items_than_grid_rows():
    """vqa_dtail_fwd / _bwd run one grid row per item (grid.y = B <= 65535): a larger batch is refused with
    VQA_E_INVALID_ARG before anything is launched (argument checks only: fake device pointers, no GPU needed)."""
    import ctypes
    lib = V.lib()
    combos = [(C, Cu, dt) for C in (32, 64) for Cu in (32, 64) for dt in (V.BF16, V.F32)
              if lib.vqa_dtail_supported(C, Cu, 4, 2, 3, 1, dt)]
    assert combos
    C, Cu, dt = combos[0]
    B, T = 70000, 8
    ws = lib.vqa_dtail_workspace(B, T, C, Cu, dt)
    p = ctypes.c_void_p(0x1000)
    rc = lib.vqa_dtail_fwd(p, p, p, p, p, p, B, T, C, Cu, dt, p, ws, None)
    assert rc == -1 and "65535" in V.last_error()
    rc = lib.vqa_dtail_bwd(p, p, p, p, p, p, p, p, p, p, p, B, T, C, Cu, dt, p, ws, None)
    assert rc == -1 and "65535" in V.last_error()
