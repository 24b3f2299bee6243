#!/bin/bash
# Spectral-kernel variants on the GPU box: per-kernel averages (rocprofv3 --stats over tools/spec_one.py) and the
# graph-timed target + loss/grad for the product library and each variant. Usage: tools/spec_ab.sh V1.so V2.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=vae-based-music--deep-generative-models_amd/libvqa.so
OUT=gpurun_out/spec_ab
mkdir -p $OUT
export TMPDIR=/tmp
cp $L $OUT/base.so
for v in $OUT/base.so "$@"; do
  cp "$v" $L
  n=$(basename $v .so)
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o t -- python tools/spec_one.py 5 > /dev/null 2>$OUT/$n.err || { cp $OUT/base.so $L; echo "$n failed"; exit 1; }
  echo "== $n: $(timeout -k 10 120 python tools/spec_one.py --time 2>/dev/null | head -1)"
  python - "$OUT/$n/t_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "spec" in r["Name"]:
        print(f"   {r['Name'][:60]:60s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
done
cp $OUT/base.so $L
