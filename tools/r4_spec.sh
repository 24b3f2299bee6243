#!/bin/bash
# Round-4 spectral pair kernel (per-pass twiddle tables, 16-padded buffers): parity tests on the new library,
# per-kernel averages of both libraries, then the step A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r4spec
mkdir -p $OUT
L=vae-based-music--deep-generative-models_amd/libvqa.so
cp $L $OUT/base.so
cp variants/spec_new.so $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_spectral.py > $OUT/tests.log 2>&1 || { cp $OUT/base.so $L; echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
for v in base new; do
  [ $v = base ] && cp $OUT/base.so $L || cp variants/spec_new.so $L
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o t -- python tools/spec_one.py 5 > /dev/null 2> $OUT/prof_$v.err || { cp $OUT/base.so $L; echo "prof $v failed"; exit 1; }
  echo "== $v: $(timeout -k 10 120 python tools/spec_one.py --time 2>/dev/null | head -1)"
  python - "$OUT/prof_$v/t_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "spec" in r["Name"]:
        print(f"   {r['Name'][:60]:60s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
done > $OUT/kernels.log 2>&1
cp $OUT/base.so $L
tools/ab_libs.sh 2 variants/spec_new.so > $OUT/step_ab.log 2>&1
