"""Per-kernel average durations (us) of gpurun_out/ktv_<variant> kernel-stats CSVs, side by side."""
import csv, glob, sys
vs = sys.argv[1:]
tabs = {}
for v in vs:
    f = max(glob.glob(f"gpurun_out/ktv_{v}/*/*_kernel_stats.csv"), key=__import__("os").path.getmtime)
    tabs[v] = {r["Name"].split("(")[0][:60]: (float(r["AverageNs"]) / 1e3, int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3)
               for r in csv.DictReader(open(f))}
names = sorted(set().union(*[set(t) for t in tabs.values()]), key=lambda n: -max(t.get(n, (0, 0, 0))[2] for t in tabs.values()))
for n in names[:int(__import__("os").environ.get("TOP", "30"))]:
    print(f"{n:60s}", "  ".join(f"{tabs[v].get(n, (0, 0, 0))[0]:9.1f}" for v in vs), "  calls", [tabs[v].get(n, (0, 0, 0))[1] for v in vs])
