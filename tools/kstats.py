#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: per kernel calls, mean µs, share (usage: kstats.py CSV [calls_per_unit])."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
per = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.3f} ms; per unit {tot / 1e3 / per:.1f} us")
for r in rows:
    print(f"{r['Name'][:96]:96s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.1f} us "
          f"{float(r['TotalDurationNs']) / 1e3 / per:8.1f} us/unit {float(r['Percentage']):5.1f}%")
