"""The shipped library's gfx950 code objects, checked on the CPU (no GPU): the build guard of DESIGN.md §5.

Kernels with packed-FP32 arithmetic (`v_pk_add_f32`, `v_pk_mul_f32`, `v_pk_fma_f32`) gave results that changed from
run to run while kernels of several hardware queues shared the CUs (profiles/r5_cotenant.txt,
profiles/r6_pk_ds_hazard.txt); `csrc/Makefile` compiles every kernel without them (`NOPK`) and runs
`csrc/check_isa.py` after the link. This test runs the same check on the library in the tree (the one the GPU box
loads): the `.hip_fatbin` section taken apart into its gfx950 code objects, each disassembled with llvm-objdump.
It also checks that the disassembly really is the product's MFMA code, so an empty or wrong-target parse cannot
pass.
"""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "vae-based-music--deep-generative-models_amd", "csrc")
LIB = os.path.join(ROOT, "vae-based-music--deep-generative-models_amd", "libvqa.so")
sys.path.insert(0, CSRC)
import check_isa  # noqa: E402


@pytest.fixture(scope="module")
def disasm():
    if not os.path.exists(LIB):
        pytest.skip("libvqa.so not built")
    if not os.path.exists(os.path.join(check_isa.LLVM, "llvm-objdump")):
        pytest.skip("llvm-objdump not in this image")
    return check_isa.disassemble(LIB)


def test_library_holds_gfx950_code_objects_per_source(disasm):
    # csrc/Makefile's SRCS: nine translation units, one bundle each
    assert len(disasm) >= 9, f"{len(disasm)} gfx950 code objects in .hip_fatbin"
    mfma = sum(len(re.findall(r"\bv_mfma_", t)) for t in disasm)
    assert mfma > 1000, f"only {mfma} MFMA instructions: not the product's kernels?"


def test_no_packed_fp32_instructions(disasm):
    hits = check_isa.packed_f32_hits(disasm)
    assert not hits, f"{len(hits)} packed-FP32 instructions (build without NOPK?): {hits[:10]}"


def test_checker_flags_packed_fp32_text():
    """The matcher itself on disassembly lines of the round-4 decoder tail (profiles/r6_pk_ds_hazard.txt)."""
    t = ("0000000000001000 <_ZN3vqa16dtail_fwd_kernel>:\n"
         "\tv_pk_add_f32 v[66:67], v[66:67], v[68:69]\n\tds_bpermute_b32 v68, v112, v66\n"
         "\tv_add_f32_e32 v1, v2, v3\n\tv_pk_fma_f32 v[0:1], v[2:3], v[4:5], v[6:7]\n\tv_pk_mul_f16 v1, v2, v3\n")
    hits = check_isa.packed_f32_hits([t])
    assert [h[1].split()[0] for h in hits] == ["v_pk_add_f32", "v_pk_fma_f32"]
    assert hits[0][0] == "_ZN3vqa16dtail_fwd_kernel"
