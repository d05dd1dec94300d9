#!/usr/bin/env python3
"""Export the per-kernel summary (rocpd `top_kernels` view) of a rocprofv3 results.db as CSV.
usage: tools/rocpd_stats.py RESULTS.db > stats.csv"""
import csv
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
cur = con.execute("select name, total_calls, total_duration, average, percentage from top_kernels")
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
for r in cur:
    w.writerow([r[0], r[1], round(r[2], 1), round(r[3], 1), round(r[4], 3)])
