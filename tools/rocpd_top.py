#!/usr/bin/env python
"""Print the per-kernel summary (calls, average us, share) from a rocprofv3 rocpd database
(the default output format): python tools/rocpd_top.py gpurun_out/<dir> [N]."""
import glob
import os
import sqlite3
import sys

db = max(glob.glob(sys.argv[1] + "/**/*.db", recursive=True), key=os.path.getmtime)
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(top_kernels)")]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
for row in c.execute("select * from top_kernels limit ?", (n,)):
    d = dict(zip(cols, row))
    name = str(d.get("name", "")).split("(")[0].replace("void ", "")[:60]
    print(f"{name:60s} {d.get('total_calls', ''):>6} {float(d.get('average', 0)):10.2f} us "
          f"{float(d.get('percentage', 0)):6.2f} %")
