#!/bin/bash
# Spectral kernels, both implementations (VQA_SPEC_IMPL=1: one wave per SIMD; default: two waves per SIMD):
# per-kernel averages (rocprofv3 --stats over tools/spec_one.py) and the graph-timed target + loss/grad.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-spec}
mkdir -p $OUT
export TMPDIR=/tmp
for impl in 1 w; do
  VQA_SPEC_IMPL=$impl timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/impl_$impl -o t -- python tools/spec_one.py 5 > /dev/null 2> $OUT/impl_$impl.err || { echo "impl $impl failed"; exit 1; }
  echo "== impl $impl: $(VQA_SPEC_IMPL=$impl timeout -k 10 120 python tools/spec_one.py --time 2>/dev/null | head -1)"
  python - "$OUT/impl_$impl/t_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "spec" in r["Name"]:
        print(f"   {r['Name'][:60]:60s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
done
