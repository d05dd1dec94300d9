#!/usr/bin/env python3
"""Per-frame timeline from a rocprofv3 kernel trace: frames start at a marker kernel; prints per frame the
span (first start to last end), the summed kernel time, the gaps, and the largest gaps with their kernels.
usage: trace_frames.py kernel_trace.csv MARKER_SUBSTRING [frame_index]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[2]
frames, cur = [], None
for r in rows:
    if marker in r["Kernel_Name"]:
        cur = []
        frames.append(cur)
    if cur is not None:
        cur.append(r)
short = lambda n: n.split("(")[0].replace("void ", "").replace("fracenc::", "")[:60]
for fi, f in enumerate(frames):
    s0, e1 = int(f[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in f)
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in f)
    print(f"frame {fi}: {len(f)} dispatches, span {(e1 - s0) / 1e3:.1f} us, kernels {busy / 1e3:.1f} us, "
          f"gaps {(e1 - s0 - busy) / 1e3:.1f} us")
want = int(sys.argv[3]) if len(sys.argv) > 3 else None
if want is not None and want < len(frames):
    f = frames[want]
    prev_end = int(f[0]["Start_Timestamp"])
    for r in f:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"  gap {(st - prev_end) / 1e3:7.1f}  dur {(en - st) / 1e3:7.1f}  {short(r['Kernel_Name'])}")
        prev_end = max(prev_end, en)
