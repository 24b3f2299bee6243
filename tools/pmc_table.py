"""Average PMC counters per dispatch of the gather kernels from rocprofv3 csv dirs (GPU dev tool).

    python tools/pmc_table.py DIR [DIR ...]
"""
import collections
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        names = {}
        for row in csv.DictReader(open(f)):
            if "gather_mfma" not in row["Kernel_Name"]:
                continue
            key = (row["Dispatch_Id"], row["Counter_Name"])
            per[key] += float(row["Counter_Value"])
            names[row["Dispatch_Id"]] = row["Kernel_Name"][:60]
        for (disp, cn), v in per.items():
            acc[names[disp]][cn].append(v)
    for k, cs in acc.items():
        print(d, k)
        for cn, vs in sorted(cs.items()):
            print(f"   {cn:28s} {sum(vs) / len(vs):16.0f}")
