#!/bin/bash
# Two PMC passes (issue / wait breakdown; instruction mix and LDS) over one program, summed per kernel whose
# name contains PATTERN (GPU dev tool). Usage: tools/pmc_kernel.sh TAG PATTERN -- python prog.py args...
set -o pipefail
TAG=$1; PAT=$2; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o p -- "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python - "$OUT" "$PAT" <<'PY'
import csv, glob, sys, collections
out, pat = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if pat not in k:
            continue
        k = k[:70]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add((f, r["Dispatch_Id"]))
for k, d in agg.items():
    print(k, "dispatch-passes", len(cnt[k]))
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {v:16.0f}")
PY
