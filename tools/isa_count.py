"""Static instruction mix of a kernel's loop body from a hipcc --save-temps .s file (dev tool).

    python tools/isa_count.py FILE.s KERNEL_SUBSTRING [--ops]

Counts MFMA / other VALU / LDS / VMEM / SALU instructions in the blocks the compiler marks as belonging to
the kernel's first outermost loop ("in Loop: Header=BB..." comments plus the header block itself), and the
register / spill numbers of the kernel's metadata.
"""
import collections
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\w+:", l) and name in l.split(":")[0]]
    if not starts:
        sys.exit(f"no kernel matching {name}")
    a = starts[0]
    sym = lines[a].split(":")[0]
    b = next(i for i in range(a, len(lines)) if ".end_amdhsa_kernel" in lines[i])
    body = lines[a:b]
    hdr = None
    for l in body:
        m = re.search(r"=>This Inner Loop Header: Depth=1", l)
        if m:
            hdr = re.match(r"^(\.LBB\w+):", l).group(1)
            break
    if hdr is None:
        sys.exit("no loop")
    key = "Header=" + hdr[2:]  # comments say Header=BB12_26
    in_loop, cur = [], False
    for i, l in enumerate(body):
        if re.match(r"^(\.LBB\w+|; %bb\.\d+):", l):
            # the block's loop comment sits on its label line or on the next line
            nxt = body[i + 1] if i + 1 < len(body) else ""
            cur = l.startswith(hdr + ":") or key in l or (key in nxt and nxt.strip().startswith(";"))
        if cur:
            in_loop.append(l)
    c, ops = collections.Counter(), collections.Counter()
    for l in in_loop:
        t = l.strip()
        if not t or t[0] in ";.":
            continue
        op = t.split()[0]
        if op.startswith("v_mfma"):
            k = "mfma"
        elif op.startswith("v_"):
            k = "valu"
        elif op.startswith("ds_"):
            k = "lds"
        elif op.startswith(("buffer_", "global_")):
            k = "vmem"
        elif op.startswith("s_"):
            k = "salu"
        else:
            k = "other"
        c[k] += 1
        ops[op] += 1
    meta = {}
    for i in range(b, len(lines)):
        if f".name:           {sym}" in lines[i] or f".symbol:         {sym}.kd" in lines[i]:
            for j in range(max(b, i - 40), min(len(lines), i + 40)):
                for k in (".vgpr_count", ".sgpr_count", ".vgpr_spill_count", ".group_segment_fixed_size"):
                    if lines[j].strip().startswith(k + ":"):
                        meta[k] = lines[j].split(":")[1].strip()
            break
    print(sym, dict(c), meta)
    if "--ops" in sys.argv:
        for op, n in ops.most_common(40):
            print(f"{n:5d} {op}")


if __name__ == "__main__":
    main()
