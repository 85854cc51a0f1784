#!/usr/bin/env python
"""Per-XCD finishing times of the tile passes (timing build: make -C csrc times).

Runs the cfg's rasterizer forward + backward several times and prints, per pass and call,
each XCD's last wave end relative to the pass's first wave start (s_memrealtime, 100 MHz),
its mean wave duration, and the makespan a perfectly balanced split of the same per-XCD
rates would have had.  GSR_STATS_DUMP=prefix also saves the raw per-tile records."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "relightable3dgaussians-w_amd")
os.environ.setdefault("GSR_LIB_PATH", os.path.join(PKG, "lib", "times", "libgsr.so"))
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402


def per_xcd(t):
    st, en, hw = t[:, 0], t[:, 1], t[:, 2]
    ok = en > 0
    t0 = st[ok].min()
    e = (en - t0) / 100.0
    d = (en - st) / 100.0
    xcc = (hw >> 32) & 0xFF
    ends, durs = [], []
    for x in range(8):
        m = ok & (xcc == x)
        ends.append(float(e[m].max()) if m.any() else 0.0)
        durs.append(float(d[m].mean()) if m.any() else 0.0)
    ends = np.array(ends)
    balanced = 8.0 / np.sum(1.0 / np.maximum(ends, 1e-9))
    return ends, durs, balanced


def main(cfg="cfg2", calls=4):
    from diff_gaussian_rasterization import _C
    from gsr import _lib, scenes
    dev = torch.device("cuda", 0)
    cam, gs, c = scenes.build_config(cfg, device="cpu", seed=0)
    g = {k: v.to(dev) for k, v in gs.items()}
    W, H, deg = cam.image_width, cam.image_height, c["sh_degree"]
    e = torch.empty(0, device=dev)
    bg = torch.zeros(3, device=dev)
    vm, pm, cp = cam.world_view_transform.to(dev), cam.full_proj_transform.to(dev), cam.camera_center.to(dev)
    L = _lib.lib()
    n = 65536  # per-unit records (GSR_UNIT_REC words each)
    tb = (C.c_ulonglong * (8 * n))()
    dout = torch.randn(3, H, W, device=dev)
    for call in range(int(calls)):
        R, color, radii, geom, binb, img = _C.rasterize_gaussians(bg, g["means3D"], e, g["opacities"], g["scales"],
                                                                  g["rotations"], 1.0, e, vm, pm, cam.tanfovx,
                                                                  cam.tanfovy, H, W, g["shs"], deg, cp, False)
        torch.cuda.synchronize()
        L.gsr_debug_fwd_times(tb, n)
        tf = np.frombuffer(tb, dtype=np.uint64).reshape(n, 8).astype(np.int64).copy()
        _C.rasterize_gaussians_backward(bg, g["means3D"], radii, e, g["scales"], g["rotations"], 1.0, e, vm, pm,
                                        cam.tanfovx, cam.tanfovy, dout, g["shs"], deg, cp, geom, R, binb, img)
        torch.cuda.synchronize()
        L.gsr_debug_bwd_times(tb, n)
        tw = np.frombuffer(tb, dtype=np.uint64).reshape(n, 8).astype(np.int64).copy()
        for name, t in (("fwd", tf), ("bwd", tw)):
            ends, durs, bal = per_xcd(t)
            print(f"call {call} {name}: makespan {ends.max():.0f} us, balanced {bal:.0f} us | ends "
                  + " ".join(f"{x:.0f}" for x in ends) + " | mean wave us " + " ".join(f"{x:.0f}" for x in durs))
            if os.environ.get("GSR_STATS_DUMP"):
                np.save(f"{os.environ['GSR_STATS_DUMP']}_{name}{call}.npy", t)


if __name__ == "__main__":
    main(*sys.argv[1:])
