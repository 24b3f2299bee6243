"""HBM traffic per launch of the dominant kernel from two rocprofv3 PMC passes (GPU dev tool).

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d DIR_F -o f -- python bench.py --no-graph --no-roofline ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d DIR_W -o w -- python bench.py --no-graph --no-roofline ...
    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d DIR_M -o m -- python bench.py ...
    python tools/pmc_traffic.py DIR_F DIR_W profiles/pmc_traffic.json [DIR_M]

FETCH_SIZE and WRITE_SIZE are in KiB. On gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane streaming
reads (MI355X_MICROARCH.md § HBM), so bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024. Both passes must
run the same workload; the per-launch figure is the mean over every dispatch of the kernel family.
MFMA busy fraction (optional third pass) = sum SQ_VALU_MFMA_BUSY_CYCLES / sum (GRBM_GUI_ACTIVE / 8 * 1024):
GRBM_GUI_ACTIVE is summed over the 8 XCDs, the busy cycles over the 1024 SIMDs (MI355X_MICROARCH.md).
"""
import csv
import glob
import json
import os
import re
import sys

FAMILY = re.compile(r"resblock_bwd_kernel(IDF16b|<__bf16|<bf16|<bool _Accum)")


def per_dispatch(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter or not FAMILY.search(row.get("Kernel_Name", "")):
                    continue
                key = (f, row.get("Dispatch_Id"))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    df, dw, out = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch = per_dispatch(df, "FETCH_SIZE")
    write = per_dispatch(dw, "WRITE_SIZE")
    if not fetch or not write:
        raise SystemExit("no dispatches of the dominant kernel found")
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    res = {"kernel": "resblock_bwd_kernel<bf16>",
           "dispatches": [len(fetch), len(write)],
           "fetch_size_kib_per_launch": round(f_kib, 1), "write_size_kib_per_launch": round(w_kib, 1),
           "per_launch_bytes": int(2 * f_kib * 1024 + w_kib * 1024),
           "note": "bytes = 2 x FETCH_SIZE (gfx950 half-count of 16-B streaming reads) + WRITE_SIZE, "
                   "mean over all dispatches of the kernel family in a --no-graph bench run"}
    if len(sys.argv) > 4:
        busy = per_dispatch(sys.argv[4], "SQ_VALU_MFMA_BUSY_CYCLES")
        grbm = per_dispatch(sys.argv[4], "GRBM_GUI_ACTIVE")
        if busy and grbm:
            res["mfma_busy_frac"] = round(sum(busy) / (sum(grbm) / 8 * 1024), 4)
            res["mfma_dispatches"] = len(busy)
    # provenance: the library these counters were read from (bench.py compares it with the library it loads)
    import hashlib
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "vae-based-music--deep-generative-models_amd", "libvqa.so")
    res["lib_sha256"] = hashlib.sha256(open(lib, "rb").read()).hexdigest() if os.path.exists(lib) else None
    res["commit"] = os.environ.get("VQA_COMMIT")  # the git HEAD the tree was sent from (no .git on the GPU box)
    import time
    res["measured_utc"] = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
