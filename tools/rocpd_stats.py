#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 results.db (rocpd): calls, total / average / median / min / max
duration in ns, percentage of the total kernel time.  The median is the figure to compare with a
kernel's timed-step mean: bench.py's pipelined host-boundary leg runs two contexts at once, and their
overlapping dispatches stretch the averages.
usage: tools/rocpd_stats.py RESULTS.db > stats.csv"""
import collections
import csv
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
d = collections.defaultdict(list)
for name, s, e in con.execute("select name, start, end from kernels"):
    d[name].append(e - s)
total = sum(sum(v) for v in d.values()) or 1
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MedianNs", "MinNs", "MaxNs", "Percentage"])
for name, v in sorted(d.items(), key=lambda x: -sum(x[1])):
    v.sort()
    w.writerow([name, len(v), sum(v), round(sum(v) / len(v), 1), v[len(v) // 2], v[0], v[-1],
                round(100.0 * sum(v) / total, 3)])
