#!/usr/bin/env python3
"""Per-launch-shape kernel durations (median of the traced launches) of the stride-2 forward convs in a
tools/kbench.py rocprofv3 --kernel-trace run per variant:  python tools/s2_trace_summary.py DIR..."""
import collections
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if "igemm" in n or "brick_x3" in n:
                key = (n.split("(")[0].replace("void mragan::", ""), int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))
                agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
        for (name, blocks), v in sorted(agg.items()):
            v.sort()
            print(f"{os.path.basename(d):10s} {name:58s} blocks {blocks:5d}  n {len(v):3d}  median {v[len(v) // 2]:7.2f} us")
