#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter values per kernel (per dispatch) from counter_collection.csv files."""
import collections
import csv
import sys

for f in sys.argv[1:]:
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        k = r["Kernel_Name"][:70]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, v in agg.items():
        if k.startswith("void at::"):
            continue
        n = len(disp[k])
        print(k, n, {c: round(x / n) for c, x in sorted(v.items())})
