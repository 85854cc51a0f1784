#!/usr/bin/env python
"""GPU-busy fraction of the bench's timed step from a rocprofv3 kernel trace: the union of all
kernel intervals (any stream) over windows of `views` consecutive k_preprocess launches in
the middle of the run, against the windows' wall length.  A fraction well below 1 means the
GPU idles between the step's kernels (host issue, synchronisation); near 1, the step is
bound by its kernels.

    python3 tools/busy.py <trace dir> [views=16]
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    views = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    f = max(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True), key=os.path.getmtime)
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0])
                  for r in csv.DictReader(open(f)))
    pre = [i for i, r in enumerate(rows) if "k_preprocess" in r[2] and "bwd" not in r[2]]
    print(f"{len(pre)} preprocess launches in {f}")
    mid = len(pre) // 2
    for a_idx in (mid - views, mid):
        if a_idx < 0 or a_idx + views >= len(pre):
            continue
        t0, t1 = rows[pre[a_idx]][0], rows[pre[a_idx + views]][0]
        iv = sorted((max(s, t0), min(e, t1)) for s, e, _ in rows if e > t0 and s < t1)
        busy, (cs, ce) = 0, iv[0]
        for s, e in iv[1:]:
            if s > ce:
                busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        print(f"views {a_idx}..{a_idx + views}: {(t1 - t0) / 1e3:.1f} us, {(t1 - t0) / views / 1e3:.1f} us per view, "
              f"GPU busy {busy / (t1 - t0):.3f}")


if __name__ == "__main__":
    main()
