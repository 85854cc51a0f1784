"""Per-kernel average durations (us) of tools/kt_variants.sh runs, side by side: for each
variant, the mean over its runs (gpurun_out/ktv_<variant>_<i>) and the spread (min-max).

    python3 tools/kt_compare.py new v5          (TOP=30 rows by default)
"""
import csv
import glob
import os
import sys


def runs(v):
    v = os.environ.get("KTP", "") + v
    out = []
    for f in sorted(glob.glob(f"gpurun_out/ktv_{v}_*/*/*_kernel_stats.csv")) + \
            sorted(glob.glob(f"gpurun_out/ktv_{v}/*/*_kernel_stats.csv")):
        out.append({r["Name"].split("(")[0][:60]: (float(r["AverageNs"]) / 1e3, int(r["Calls"]),
                                                   float(r["TotalDurationNs"]) / 1e3) for r in csv.DictReader(open(f))})
    return out


vs = sys.argv[1:]
tabs = {v: runs(v) for v in vs}
names = sorted(set().union(*[set(t) for rs in tabs.values() for t in rs]),
               key=lambda n: -max(t.get(n, (0, 0, 0))[2] for rs in tabs.values() for t in rs))
print(f"{'kernel':60s}", "  ".join(f"{v:>22s}" for v in vs))
for n in names[:int(os.environ.get("TOP", "30"))]:
    cells = []
    for v in vs:
        a = [t[n][0] for t in tabs[v] if n in t]
        cells.append(f"{sum(a) / len(a):8.1f} ({min(a):6.1f}-{max(a):6.1f})" if a else f"{'-':>22s}")
    print(f"{n:60s}", "  ".join(cells))
