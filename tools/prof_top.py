"""Per-step kernel breakdown from a rocprofv3 --kernel-trace SQLite DB (rocpd; durations in us): python tools/prof_top.py DB [steps]."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = db.execute("select name, total_calls, total_duration, average from top_kernels").fetchall()
tot = sum(r[2] for r in rows)
print(f"total {tot / 1e3 / steps:.3f} ms/step over {steps:g} steps")
for name, calls, dur, avg in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    short = name if len(name) < 90 else name[:87] + "..."
    print(f"{dur / 1e3 / steps:8.3f} ms {calls / steps:7.1f}/step avg {avg:8.2f} us  {short}")
