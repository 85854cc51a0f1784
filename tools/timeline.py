#!/usr/bin/env python
"""Per-kernel timeline of one rasterizer call pair from a rocprofv3 kernel trace (csv):
start offset, duration and the idle gap before each kernel, for the LAST complete window
that starts at a preprocess launch.  python tools/timeline.py <trace dir> [first-kernel-prefix]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else "k_preprocess_regsh"
f = max(glob.glob(d + "/**/*kernel_trace.csv", recursive=True), key=os.path.getmtime)
rows = []
with open(f) as fh:
    for r in csv.DictReader(fh):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]
                     .replace("void ", "").replace("gsr::", "")))
rows.sort()
starts = [i for i, r in enumerate(rows) if r[2].startswith(first)]
a, b = starts[-3], starts[-2]
t0 = rows[a][0]
prev_end = t0
tot_gap = tot_busy = 0
for s, e, n in rows[a:b]:
    gap = s - prev_end
    tot_gap += max(gap, 0)
    tot_busy += e - s
    print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {gap / 1e3:6.1f}  {n[:70]}")
    prev_end = max(prev_end, e)
print(f"window {(rows[b][0] - t0) / 1e3:.1f} us, busy {tot_busy / 1e3:.1f} us, gaps {tot_gap / 1e3:.1f} us, "
      f"{b - a} kernels")
