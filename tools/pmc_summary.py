#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel (average per dispatch)."""
import collections
import csv
import sys

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, v in agg.items():
        n = len(disp[k])
        print(f"{k} [{n} dispatches]")
        for c, val in sorted(v.items()):
            print(f"    {c:32s} {val / n:.4g}")
