"""Per-step kernel breakdown from a rocprofv3 kernel_trace.csv (GPU dev tool): takes the interval between two
consecutive adam_kernel dispatches (one train step) in the middle of the run and groups kernel time.

    python tools/step_breakdown.py KERNEL_TRACE_CSV [STEP_INDEX]
"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(adam) // 2
a, b = adam[k], adam[k + 1]
step = rows[a + 1:b + 1]
wall = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e6
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step) / 1e6
print(f"step {k}: {len(step)} dispatches, wall {wall:.3f} ms, kernel-busy {busy:.3f} ms")
# concurrent streams: time with >= 1 kernel running, and the busy time of each queue / stream
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step)
union, cur_s, cur_e = 0, iv[0][0], iv[0][1]
for s0, e0 in iv[1:]:
    if s0 > cur_e:
        union += cur_e - cur_s
        cur_s, cur_e = s0, e0
    else:
        cur_e = max(cur_e, e0)
union += cur_e - cur_s
print(f"  GPU busy (>= 1 kernel) {union / 1e6:.3f} ms, idle {wall - union / 1e6:.3f} ms")
for col in ("Stream_Id", "Queue_Id"):
    if col in step[0]:
        per = collections.defaultdict(float)
        for r in step:
            per[r[col]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        print(f"  per {col}: " + ", ".join(f"{q}: {t:.3f} ms" for q, t in sorted(per.items())))
by = collections.defaultdict(lambda: [0, 0.0])
for r in step:
    n = r["Kernel_Name"]
    key = n.split("(")[0][:90] + f"  grid={r['Grid_Size_X']}"
    if len(sys.argv) > 3:
        key = n[:100]
    by[key][0] += 1
    by[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for key, (c, t) in sorted(by.items(), key=lambda kv: -kv[1][1])[:60]:
    print(f"{t:8.3f} ms {c:5d}x  {key}")
