#!/usr/bin/env python
"""Per-unit timeline of the tile passes (timing build: make -C csrc times).

Every workgroup of k_render_fwd / k_render_bwd that takes a unit (a whole tile or one
quadrant of a split tile) records its start / end (s_memrealtime, 100 MHz), hardware id,
tile, quadrant mask, cost estimate and work count.  Prints per pass: makespan, the number of
whole / split units, the longest units (duration, start, cost), and what ends the pass (the
units finishing in its last 10 %).  GSR_STATS_DUMP=prefix saves the raw records (.npy).

  python tools/unit_times.py [cfg2c] [calls]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "relightable3dgaussians-w_amd")
os.environ.setdefault("GSR_LIB_PATH", os.path.join(PKG, "lib", "times", "libgsr.so"))
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402

REC = 8
MAXU = 65536


def analyse(name, t):
    ok = t[:, 1] > 0
    t = t[ok]
    st, en = t[:, 0], t[:, 1]
    t0 = st.min()
    d = (en - st) / 100.0
    s = (st - t0) / 100.0
    e = (en - t0) / 100.0
    span = e.max()
    whole = t[:, 4] == 15
    print(f"  {name}: makespan {span:.1f} us, units {len(t)} ({whole.sum()} whole, {(~whole).sum()} quadrant), "
          f"wave us p50 {np.median(d):.1f} p90 {np.percentile(d, 90):.1f} max {d.max():.1f}, sum {d.sum():.0f}")
    o = np.argsort(-d)[:6]
    print("    longest (us, start, tile, qmask, cost, work): " +
          "; ".join(f"{d[i]:.0f} @{s[i]:.0f} t{t[i, 3]} q{t[i, 4]} c{t[i, 5]} w{t[i, 6]}" for i in o))
    late = e >= 0.9 * span
    print(f"    ending in the last 10 %: {late.sum()} units, their starts p10/p50/max "
          f"{np.percentile(s[late], 10):.0f}/{np.median(s[late]):.0f}/{s[late].max():.0f} us, durations p50/max "
          f"{np.median(d[late]):.0f}/{d[late].max():.0f}; last start {s.max():.0f} us")
    # how busy the chip is over time: units in flight per 5 % of the makespan
    edges = np.linspace(0, span, 21)
    infl = [int(((s <= x) & (e > x)).sum()) for x in edges[:-1]]
    print("    units in flight per 5 %: " + " ".join(str(v) for v in infl))


def main(cfg="cfg2c", calls=3):
    from diff_gaussian_rasterization import _C
    from gsr import _lib, scenes
    dev = torch.device("cuda", 0)
    cam, gs, c = scenes.build_config(cfg, device="cpu", seed=0)
    g = {k: v.to(dev) for k, v in gs.items() if k != "is_sky"}
    W, H, deg = cam.image_width, cam.image_height, c["sh_degree"]
    e = torch.empty(0, device=dev)
    bg = torch.zeros(3, device=dev)
    vm, pm, cp = cam.world_view_transform.to(dev), cam.full_proj_transform.to(dev), cam.camera_center.to(dev)
    L = _lib.lib()
    tb = (C.c_ulonglong * (REC * MAXU))()
    dout = torch.randn(3, H, W, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    for call in range(int(calls)):
        L.gsr_debug_fwd_times_reset()
        L.gsr_debug_bwd_times_reset()
        L.gsr_debug_st_times_reset()
        torch.cuda.synchronize()
        R, color, radii, geom, binb, img = _C.rasterize_gaussians(bg, g["means3D"], e, g["opacities"], g["scales"],
                                                                  g["rotations"], 1.0, e, vm, pm, cam.tanfovx,
                                                                  cam.tanfovy, H, W, g["shs"], deg, cp, False)
        _C.rasterize_gaussians_backward(bg, g["means3D"], radii, e, g["scales"], g["rotations"], 1.0, e, vm, pm,
                                        cam.tanfovx, cam.tanfovy, dout, g["shs"], deg, cp, geom, R, binb, img)
        torch.cuda.synchronize()
        print(f"{cfg} call {call}")
        sb = (C.c_ulonglong * (4 * MAXU))()
        L.gsr_debug_st_times(sb, MAXU)
        t = np.frombuffer(sb, dtype=np.uint64).reshape(MAXU, 4).astype(np.int64).copy()
        t = t[t[:, 2] > 0]
        if len(t):
            t0 = t[:, 0].min()
            setup = (t[:, 1] - t[:, 0]) / 100.0
            pas = (t[:, 2] - t[:, 1]) / 100.0
            end = (t[:, 2] - t0) / 100.0
            o = np.argsort(-pas)[:5]
            print(f"  st_scatter: span {end.max():.1f} us over {len(t)} waves; set-up p50/max {np.median(setup):.1f}/"
                  f"{setup.max():.1f} us; ranking pass p50/p99/max {np.median(pas):.1f}/{np.percentile(pas, 99):.1f}/"
                  f"{pas.max():.1f} us; longest passes (us, block, start): "
                  + "; ".join(f"{pas[i]:.0f} b{t[i, 3]} @{(t[i, 1] - t0) / 100:.0f}" for i in o))
            if os.environ.get("GSR_STATS_DUMP"):
                np.save(f"{os.environ['GSR_STATS_DUMP']}_st{call}.npy", t)
        for name, fn in (("fwd", L.gsr_debug_fwd_times), ("bwd", L.gsr_debug_bwd_times)):
            fn(tb, MAXU)
            t = np.frombuffer(tb, dtype=np.uint64).reshape(MAXU, REC).astype(np.int64).copy()
            analyse(name, t)
            if os.environ.get("GSR_STATS_DUMP"):
                np.save(f"{os.environ['GSR_STATS_DUMP']}_{name}{call}.npy", t[t[:, 1] > 0])


if __name__ == "__main__":
    main(*sys.argv[1:])
