#!/usr/bin/env python
"""Where the cfg4 training iteration spends GPU time outside the HIP kernels: runs a few
train_step()s under torch.profiler and prints the device-time table grouped by Python
call site (tools only; run on the GPU box).

    python tools/train_glue.py [P_fg] [rows]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd")]

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def main():
    from gsr import train
    P_fg = int(sys.argv[1]) if len(sys.argv) > 1 else 1_363_637
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    dev = torch.device("cuda", 0)
    scene, views, gts = train.synthetic_relit_scene(P_fg, 4, 1920, 1080, 1400.0, dev, seed=0)
    scene.iteration = train.REG_NORMAL_FROM_ITER  # every loss term on, as bench.py's train leg
    ids = list(range(4))
    for _ in range(3):
        train.train_step(scene, views, ids, gts)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof:
        for _ in range(3):
            train.train_step(scene, views, ids, gts)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="device_time_total", row_limit=rows, max_name_column_width=60))
    # the PyTorch glue by input shapes (which tensors the copies, products, sums and fills run on)
    ka = prof.key_averages(group_by_input_shape=True)
    glue = [e for e in ka if e.key.startswith("aten::") and e.device_time_total > 0]
    glue.sort(key=lambda e: -e.device_time_total)
    print("\n%-28s %10s %6s  %s" % ("op", "device us", "calls", "input shapes"))
    for e in glue[:rows]:
        print("%-28s %10.1f %6d  %s" % (e.key, e.device_time_total, e.count, str(e.input_shapes)[:150]))
    # ... and by Python call site (the innermost frames in this repository)
    ks = prof.key_averages(group_by_stack_n=8)
    sites = {}
    top = sorted([e for e in ks if e.key.startswith("aten::")], key=lambda e: -e.device_time_total)[:2]
    for e in top:
        print("stack sample:", e.key, e.stack[:10])
    for e in ks:
        if not e.key.startswith("aten::") or e.device_time_total <= 0:
            continue
        fr = [f for f in (e.stack or []) if "relightable3dgaussians-w_amd" in f or "/repo/" in f]
        site = " < ".join(f.split("/")[-1] for f in fr[:3]) or "?"
        d = sites.setdefault(site, [0.0, 0, set()])
        d[0] += e.device_time_total
        d[1] += e.count
        d[2].add(e.key)
    print("\n%10s %6s  %s" % ("device us", "calls", "call site (ops)"))
    for site, (t, n, ops) in sorted(sites.items(), key=lambda kv: -kv[1][0])[:rows]:
        print("%10.1f %6d  %s  (%s)" % (t, n, site[:160], ",".join(sorted(o[6:] for o in ops))[:80]))


if __name__ == "__main__":
    main()
