#!/usr/bin/env python
"""Turn one round's rocprofv3 outputs (tools/profile_round.sh) into the committed evidence under
profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_hbm_traffic.json   per kernel: calls, avg duration, FETCH_SIZE / WRITE_SIZE per
                                    launch and the corrected HBM bytes per launch
  profiles/<tag>_summary.md         the same as a table, plus the bench line printed under the
                                    profiler (its stage_ms must agree with the kernel averages)

HBM correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE/WRITE_SIZE are KiB; on gfx950
FETCH_SIZE reports 1/2 of the bytes of wide streaming reads, so
    traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024  bytes per launch.
The factor is calibrated for 16-B-per-lane streaming loads; gathers of 48-B records are not
calibrated, so the read half is an estimate (ratios between kernel variants are exact).
"""
import csv
import glob
import json
import os
import statistics
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.split("(")[0].replace("gsr::", "").replace("void ", "")


def newest_run(files):
    """The files of the newest rocprofv3 run among files (gpurun_out/ keeps earlier calls' runs of
    the same tag beside it: <pid>_*.csv, one pid per run)."""
    if not files:
        return []
    last = max(files, key=os.path.getmtime)
    pid = os.path.basename(last).split("_")[0]
    return [f for f in files if os.path.dirname(f) == os.path.dirname(last) and os.path.basename(f).split("_")[0] == pid]


def counters(pattern):
    acc = defaultdict(list)
    for f in newest_run(glob.glob(pattern)):
        for r in csv.DictReader(open(f)):
            acc[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return acc


def main(tag="r01", workload=None):
    out_dir = os.path.join(ROOT, "profiles")
    os.makedirs(out_dir, exist_ok=True)
    g = os.path.join(ROOT, "gpurun_out")
    ks = newest_run(glob.glob(os.path.join(g, f"prof_{tag}_kt", "*", "*_kernel_stats.csv")))
    if not ks:
        sys.exit(f"no kernel stats for {tag}")
    rows = list(csv.DictReader(open(ks[-1])))
    with open(os.path.join(out_dir, f"{tag}_kernel_stats.csv"), "w") as f:
        f.write(open(ks[-1]).read())
    fetch = counters(os.path.join(g, f"prof_{tag}_fetch", "*", "*_counter_collection.csv"))
    write = counters(os.path.join(g, f"prof_{tag}_write", "*", "*_counter_collection.csv"))
    valu = counters(os.path.join(g, f"prof_{tag}_valu", "*", "*_counter_collection.csv"))
    res = {}
    for r in rows:
        k = short(r["Name"])
        fr = fetch.get((k, "FETCH_SIZE"))
        wr = write.get((k, "WRITE_SIZE"))
        fk = statistics.mean(fr) if fr else None
        wk = statistics.mean(wr) if wr else None
        vi = valu.get((k, "SQ_INSTS_VALU"))
        si = valu.get((k, "SQ_INSTS_SALU"))
        wv = valu.get((k, "SQ_WAVES"))
        res[k] = dict(calls=int(r["Calls"]), avg_ms=float(r["AverageNs"]) / 1e6, pct=float(r["Percentage"]),
                      fetch_kib=fk, write_kib=wk,
                      traffic_bytes=(None if fk is None or wk is None else (2 * fk + wk) * 1024.0),
                      valu_insts=statistics.mean(vi) if vi else None, salu_insts=statistics.mean(si) if si else None,
                      waves=statistics.mean(wv) if wv else None)
    bench = None
    log = os.path.join(g, f"prof_{tag}_kt.log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{\"metric\""):
                bench = json.loads(line)
    json.dump(dict(tag=tag, created=time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
                   correction="traffic = (2*FETCH_SIZE + WRITE_SIZE) * 1024 B per launch (gfx950)",
                   command=("tools/profile_train.sh: rocprofv3 --kernel-trace --stats, then separate --pmc FETCH_SIZE, "
                            "--pmc WRITE_SIZE, --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES passes over "
                            "tools/train_kernels.py") if workload else
                           ("rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 10 --warmup 3 "
                           "--no-cpu-baseline --no-refalgo --no-train [--no-minibatch] <workload args>; separate "
                           "--pmc FETCH_SIZE, --pmc WRITE_SIZE and --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES passes"),
                   workload=workload, kernels=res, bench_under_profiler=bench),
              open(os.path.join(out_dir, f"{tag}_hbm_traffic.json"), "w"), indent=1)
    with open(os.path.join(out_dir, f"{tag}_summary.md"), "w") as f:
        wl = workload or ((bench or {}).get("config") or {}).get("workload", "bench.py's default workload")
        f.write(f"# rocprofv3 summary {tag}\n\n{'tools/profile_train.sh' if workload else 'bench.py'} under "
                f"rocprofv3, workload: {wl}; "
                "traffic = (2*FETCH_SIZE + WRITE_SIZE)*1024 B per launch.\n\n")
        f.write("| kernel | calls | avg ms | % | FETCH KiB | WRITE KiB | HBM MB/launch | GB/s | VALU Minst/launch "
                "| SALU Minst/launch |\n|---|---|---|---|---|---|---|---|---|---|\n")
        for k, v in sorted(res.items(), key=lambda kv: -kv[1]["pct"]):
            tb = v["traffic_bytes"]
            f.write(f"| {k} | {v['calls']} | {v['avg_ms']:.4f} | {v['pct']:.1f} | "
                    f"{'' if v['fetch_kib'] is None else round(v['fetch_kib'])} | "
                    f"{'' if v['write_kib'] is None else round(v['write_kib'])} | "
                    f"{'' if tb is None else round(tb / 1e6, 2)} | "
                    f"{'' if tb is None else round(tb / (v['avg_ms'] * 1e-3) / 1e9, 1)} | "
                    f"{'' if v['valu_insts'] is None else round(v['valu_insts'] / 1e6, 2)} | "
                    f"{'' if v['salu_insts'] is None else round(v['salu_insts'] / 1e6, 2)} |\n")
        if bench:
            f.write(f"\nbench line under the profiler: value {bench['value']} {bench.get('unit', 'MPix/s')}, ms/step {bench['ms_per_step']}"
                    f"\n\nstage_ms (HIP events): {json.dumps(bench.get('stage_ms'))}\n")
    print(open(os.path.join(out_dir, f"{tag}_summary.md")).read())


if __name__ == "__main__":
    main(*sys.argv[1:])
