"""Compare the disassembled machine code of kernels between two libvqa.so builds (dev tool).
    python tools/kernel_diff.py OLD.so NEW.so REGEX
Prints, per kernel symbol matching REGEX (in either library), whether its instruction stream is identical (addresses
and branch-target labels stripped), or its instruction counts."""
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "vae-based-music--deep-generative-models_amd", "csrc"))
import check_isa  # noqa: E402


def funcs(lib):
    out = {}
    for t in check_isa.disassemble(lib):
        cur = None
        for line in t.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:", line)
            if m:
                cur = m.group(1)
                out[cur] = []
                continue
            if cur is None:
                continue
            ins = line.split("//")[0].strip()
            if not ins or ins.startswith(";"):
                continue
            ins = re.sub(r"<[^>]*>", "<L>", ins)
            ins = re.sub(r"\b0x[0-9a-f]+\b(?=\s*$)", "", ins)
            out[cur].append(ins)
    return out


def main():
    old, new, rx = sys.argv[1], sys.argv[2], re.compile(sys.argv[3])
    a, b = funcs(old), funcs(new)
    for name in sorted(set(a) | set(b)):
        if not rx.search(name):
            continue
        x, y = a.get(name), b.get(name)
        if x is None or y is None:
            print(f"{'only new' if x is None else 'only old':10s} {name}")
        elif x == y:
            print(f"{'same':10s} {name} ({len(x)} instructions)")
        else:
            def cnt(v):
                c = {"mfma": 0, "valu": 0, "lds": 0, "vmem": 0, "salu": 0}
                for i in v:
                    op = i.split()[0]
                    k = ("mfma" if op.startswith("v_mfma") else "valu" if op.startswith("v_") else "lds"
                         if op.startswith("ds_") else "vmem" if op.startswith(("buffer_", "global_")) else "salu")
                    c[k] += 1
                return c
            print(f"{'differs':10s} {name}: old {cnt(x)} new {cnt(y)}")


if __name__ == "__main__":
    main()
