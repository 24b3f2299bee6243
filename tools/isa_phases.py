"""Instruction mix of a kernel between phase markers (dev tool): build a copy of the source with RS_STAMP(i) defined
as `asm volatile(";RSMARK i")` and --save-temps, then
    python tools/isa_phases.py FILE.s KERNEL_SUBSTRING
counts, per stretch of code that follows a marker (up to the next marker), MFMA / VALU by class / LDS / VMEM /
SALU instructions. VALU classes: arith (f32 add/mul/fma/max/min), cvt (bf16 <-> f32 conversions, packed converts),
mask (packed u16/i16 ops on bf16 bits), select (v_cndmask, v_cmp), addr (integer add/shift/and/or/lshl_add/mad on
addresses and indices), move (v_mov, v_readfirstlane, accvgpr moves).
"""
import collections
import re
import sys


def vclass(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_cndmask", "v_cmp")):
        return "select"
    if op.startswith(("v_cvt",)):
        return "cvt"
    if op.startswith(("v_pk_max_i16", "v_pk_min_u16", "v_pk_mul_lo_u16", "v_pk_max_u16", "v_pk_min_i16")):
        return "mask"
    if op.startswith(("v_add_f32", "v_sub_f32", "v_mul_f32", "v_fma_f32", "v_max_f32", "v_min_f32", "v_pk_add_f32",
                      "v_pk_mul_f32", "v_pk_fma_f32")):
        return "arith"
    if op.startswith(("v_mov", "v_readfirstlane", "v_accvgpr", "v_readlane", "v_writelane")):
        return "move"
    if op.startswith(("v_lshl", "v_lshr", "v_ashr", "v_and", "v_or", "v_xor", "v_add_u", "v_add_i", "v_sub_u",
                      "v_sub_i", "v_mad_u", "v_mad_i", "v_mul_lo", "v_mul_hi", "v_bfe", "v_bfi", "v_perm", "v_add3",
                      "v_lshl_add", "v_lshl_or", "v_and_or", "v_or3", "v_xad", "v_alignbit", "v_add_co", "v_sub_co",
                      "v_addc", "v_subb", "v_mul_u32", "v_min_i32", "v_max_i32", "v_min_u32", "v_max_u32",
                      "v_not")):
        return "addr"
    return "valu_other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\w+:", l) and name in l.split(":")[0]]
    if not starts:
        sys.exit(f"no kernel matching {name}")
    a = starts[0]
    b = next(i for i in range(a, len(lines)) if ".end_amdhsa_kernel" in lines[i])
    cur = "prologue"
    seen = []
    counts = collections.OrderedDict()
    ops = collections.defaultdict(collections.Counter)
    for l in lines[a:b]:
        m = re.search(r";RSMARK (\d+)", l)
        if m:
            cur = f"after mark {m.group(1)}"
            seen.append(cur)
            continue
        t = l.strip()
        if not t or t[0] in ";." or t.endswith(":"):
            continue
        op = t.split()[0]
        if op.startswith("v_"):
            k = vclass(op)
        elif op.startswith("ds_"):
            k = "lds"
        elif op.startswith(("buffer_", "global_")):
            k = "vmem"
        elif op.startswith("s_"):
            k = "salu"
        else:
            k = "other"
        counts.setdefault(cur, collections.Counter())[k] += 1
        ops[cur][op] += 1
    keys = ["mfma", "arith", "cvt", "mask", "select", "addr", "move", "valu_other", "lds", "vmem", "salu"]
    print(f"{'stretch':16s} " + " ".join(f"{k:>6s}" for k in keys) + "   VALU")
    tot = collections.Counter()
    for st, c in counts.items():
        valu = sum(c[k] for k in keys[1:8])
        tot.update(c)
        print(f"{st:16s} " + " ".join(f"{c[k]:6d}" for k in keys) + f"  {valu:5d}")
    valu = sum(tot[k] for k in keys[1:8])
    print(f"{'total':16s} " + " ".join(f"{tot[k]:6d}" for k in keys) + f"  {valu:5d}")
    if "--ops" in sys.argv:
        for st, c in ops.items():
            print(st, dict(c.most_common(25)))


if __name__ == "__main__":
    main()
