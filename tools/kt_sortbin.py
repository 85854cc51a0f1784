"""Depth-sort and binning kernel averages (us) of gpurun_out/<prefix>_* kernel traces, one line
per run, plus the bench's ms_per_step.  python tools/kt_sortbin.py kt46"""
import csv, glob, json, os, re, sys

pre = sys.argv[1]
for d in sorted(glob.glob(f"gpurun_out/{pre}_*"), key=lambda x: int((re.findall(r"_(\d+)_", x) or ["0"])[0])):
    if d.endswith(".log") or not re.search(r"_\d+_", d):
        continue
    fs = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)
    if not fs:
        continue
    t = {r["Name"].split("(")[0]: (float(r["AverageNs"]) / 1e3, int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3)
         for r in csv.DictReader(open(fs[0]))}
    calls = max(v[1] for k, v in t.items() if "render_fwd" in k)
    per_call = lambda pat: sum(v[2] for k, v in t.items() if pat in k) / calls
    ms = re.findall(r'"ms_per_step": ([0-9.]+)', open(d + ".log").read())
    print(f"{os.path.basename(d):22s} sort {per_call('radix_scatter') + per_call('radix_hist'):6.1f}  scatter passes "
          f"{[round(v[0], 1) for k, v in sorted(t.items()) if 'radix_scatter' in k]}  st_hist {per_call('k_st_hist'):5.1f}  "
          f"st_scatter {per_call('k_st_scatter'):6.1f}  ms/step {ms[0] if ms else '-'}")
