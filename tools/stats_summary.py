"""Summarise a rocprofv3 --stats kernel_stats.csv: top kernels and the dominant kernel family's combined
average (all conv32_kernel<bf16, ...> instantiations), for profiles/.

    python tools/stats_summary.py KERNEL_STATS_CSV [BENCH_JSON [BENCH_JSON_DEFAULT]] > profiles/rNN_summary.md
"""
import csv
import json
import re
import sys

FAMILY = re.compile(r"resblock_bwd_kernel(IDF16b|<__bf16|<bf16|<bool _Accum)")
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"# rocprofv3 --kernel-trace --stats summary ({sys.argv[1].split('/')[-1]})\n")
print("| kernel | calls | total ms | avg us | % |\n|---|---|---|---|---|")
for r in rows[:20]:
    n = r["Name"] if len(r["Name"]) < 100 else r["Name"][:97] + "..."
    print(f"| `{n}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['AverageNs']) / 1e3:.2f} "
          f"| {float(r['Percentage']):.1f} |")
fam = [r for r in rows if FAMILY.search(r["Name"])]
calls = sum(int(r["Calls"]) for r in fam)
dur = sum(float(r["TotalDurationNs"]) for r in fam)
print(f"\nDominant kernel resblock_bwd_kernel<bf16> ({len(fam)} instantiations): "
      f"{calls} calls, average {dur / max(calls, 1) / 1e3:.2f} us, {100 * dur / tot:.1f} % of kernel time.")
if len(sys.argv) > 2:
    b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    r = b["roofline"]
    print(f"\nbench.py line of the same (levels serialised, VQA_LEVEL_STREAMS=0) run: {b['ms_per_step']} ms/step, {b['value'] / 1e6:.2f} M {b['unit']}; "
          f"roofline avg_launch_us {r['avg_launch_us']}, achieved {r['achieved']} GB/s "
          f"({100 * r['frac']:.1f} % of {r['peak']}), traffic {r['traffic']} B/launch vs algorithmic "
          f"{r['algorithmic_bytes_per_launch']} B/launch.")
if len(sys.argv) > 3:
    b = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
    r = b["roofline"]
    print(f"\nbench.py line with default settings (levels on concurrent streams), no profiler: "
          f"{b['ms_per_step']} ms/step, {b['value'] / 1e6:.2f} M {b['unit']}; roofline avg_launch_us "
          f"{r['avg_launch_us']} ({100 * r['frac']:.1f} % of {r['peak']} {r['unit']}).")
