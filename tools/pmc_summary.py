"""Summarise rocprofv3 --pmc CSVs: mean counter value per (kernel, counter), plus derived ratios."""
import collections
import csv
import glob
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc01_*/*/*_counter_collection.csv"
acc = collections.defaultdict(list)
for f in glob.glob(pat):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("gsr::", "")
        acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
kern = sorted({k for k, _ in acc})
ctrs = sorted({c for _, c in acc})
for k in kern:
    vals = {c: sum(acc[(k, c)]) / len(acc[(k, c)]) for c in ctrs if (k, c) in acc}
    print(f"== {k}")
    for c, v in vals.items():
        print(f"   {c:28s} {v:16.1f}")
    w = vals.get("SQ_WAVES")
    if w:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD"):
            if c in vals:
                print(f"   {c + '/wave':28s} {vals[c] / w:16.1f}")
    if "SQ_WAVE_CYCLES" in vals and "SQ_WAIT_ANY" in vals:
        wc = vals["SQ_WAVE_CYCLES"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS",
                  "SQ_ACTIVE_INST_LDS"):
            if c in vals:
                print(f"   {c + ' / WAVE_CYCLES':40s} {vals[c] / wc:8.3f}")
    if "SQ_THREAD_CYCLES_VALU" in vals and "SQ_ACTIVE_INST_VALU" in vals:
        print(f"   {'VALU lane utilisation':40s} {vals['SQ_THREAD_CYCLES_VALU'] / (vals['SQ_ACTIVE_INST_VALU'] * 64):8.3f}")
