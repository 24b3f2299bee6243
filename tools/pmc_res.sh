#!/bin/bash
# PMC passes over the fused residual-block kernels (GPU dev tool). Usage: tools/pmc_res.sh TAG
set -o pipefail
TAG=${1:-pmcres}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o p -- python tools/resblock_one.py ${WHICH:-both} ${T:-32768} ${DIL:-9} 3 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = "fwd" if "fwd" in r["Kernel_Name"] else ("bwd" if "bwd" in r["Kernel_Name"] else None)
        if not k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add((f, r["Dispatch_Id"]))
for k, d in agg.items():
    print(k, "dispatch-passes", len(cnt[k]))
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {v:16.0f}")
PY
