#!/usr/bin/env python
"""Work counters of the tile passes at cfg2 (instrumented build: make -C csrc stats).

Prints per-tile averages: list entries examined, survivors of the quadrant culling,
(Gaussian, quadrant) evaluations, evaluations with at least one contributing lane, and the
mean number of contributing lanes per such evaluation."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "relightable3dgaussians-w_amd")
os.environ["GSR_LIB_PATH"] = os.path.join(PKG, "lib", "stats", "libgsr.so")
sys.path[:0] = [ROOT, PKG]

import torch  # noqa: E402


def main(cfg="cfg2"):
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
    buf = (C.c_ulonglong * 8)()
    L.gsr_debug_fwd_stats(buf, 1)
    L.gsr_debug_bwd_stats(buf, 1)
    R, color, radii, geom, binb, img = _C.rasterize_gaussians(bg, g["means3D"], e, g["opacities"], g["scales"],
                                                              g["rotations"], 1.0, e, vm, pm, cam.tanfovx,
                                                              cam.tanfovy, H, W, g["shs"], deg, cp, False)
    dout = torch.randn(3, H, W, device=dev)
    _C.rasterize_gaussians_backward(bg, g["means3D"], radii, e, g["scales"], g["rotations"], 1.0, e, vm, pm,
                                    cam.tanfovx, cam.tanfovy, dout, g["shs"], deg, cp, geom, R, binb, img)
    torch.cuda.synchronize()
    T = ((W + 15) // 16) * ((H + 15) // 16)
    out = {"R": int(R), "tiles": T}
    for name, fn in (("fwd", L.gsr_debug_fwd_stats), ("bwd", L.gsr_debug_bwd_stats)):
        fn(buf, 1)
        v = [int(x) for x in buf]
        out[name] = {"entries_per_tile": v[0] / T, "survivors_per_tile": v[1] / T, "quad_evals_per_tile": v[2] / T,
                     "quad_evals_with_work_per_tile": v[3] / T,
                     "lanes_per_working_eval": v[4] / max(v[3], 1),
                     "gaussians_with_work_per_tile": (v[5] / T) if name == "bwd" else None,
                     "survivors_reaching_all_quadrants": (v[5] / max(v[6], 1)) if name == "fwd" else None,
                     "queue_wait_us_total": v[6] / 100.0 if name == "bwd" else None,
                     "tiles_via_queue": v[7] if name == "bwd" else None}
    n = 65536  # per-unit records (GSR_UNIT_REC words each)
    tb = (C.c_ulonglong * (8 * n))()
    import numpy as np
    if os.environ.get("GSR_STATS_DUMP"):
        L.gsr_debug_fwd_times(tb, n)
        np.save(os.environ["GSR_STATS_DUMP"] + "_fwd.npy", np.frombuffer(tb, dtype=np.uint64).reshape(n, 8).astype(np.int64))
    L.gsr_debug_bwd_times(tb, n)
    t = np.frombuffer(tb, dtype=np.uint64).reshape(n, 8).astype(np.int64)
    t = t[t[:, 1] > 0]
    st, en, hw = t[:, 0], t[:, 1], t[:, 2]
    if os.environ.get("GSR_STATS_DUMP"):
        np.save(os.environ["GSR_STATS_DUMP"] + "_bwd.npy", t)
    dur = (en - st) / 100.0  # s_memrealtime: 100 MHz -> us
    span = (en.max() - st.min()) / 100.0
    hwid = hw & 0xffffffff
    simd = ((hwid >> 4) & 3) | (((hwid >> 8) & 15) << 2) | (((hwid >> 12) & 1) << 6) | (((hwid >> 13) & 7) << 7) | ((hw >> 32) << 10)
    _, counts = np.unique(simd, return_counts=True)
    rel0 = (st - st.min()) / 100.0
    out["bwd_timing"] = {"makespan_us": span, "wave_us_mean": float(dur.mean()), "wave_us_p50": float(np.median(dur)),
                         "wave_us_p99": float(np.percentile(dur, 99)), "wave_us_max": float(dur.max()),
                         "sum_wave_us": float(dur.sum()), "distinct_simds": int(len(counts)),
                         "waves_per_simd_max": int(counts.max()), "waves_per_simd_mean": float(counts.mean()),
                         "last_start_us": float(rel0.max()), "start_p90_us": float(np.percentile(rel0, 90))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
