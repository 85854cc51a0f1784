#!/usr/bin/env python
"""Pixels whose n_contrib differs between the GPU forward and the C oracle, replayed on the CPU:
for each, the contributions near the end of its list with the oracle's alpha (float32, the
reference's operation order, expf via float64), the tile passes' p' and alpha (gsr_tile.hpp
gauss_lpower emulated with float64-rounded FMAs), the record's guard band eps_r and the
transmittance -- which decision flipped and why.

    python tools/diag_decisions.py [case names...]   (tests/test_gpu_rasterizer.py CASES)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd")]

f32 = np.float32


def fma(a, b, c):
    return f32(np.float64(a) * np.float64(b) + np.float64(c))


def replay(rec, pl, rg, tile, px, py, nc_gpu, nc_ref, show=6):
    lo, hi = int(rg[tile, 0]), int(rg[tile, 1])
    T = f32(1.0)
    rows = []
    LOG2E = f32(1.44269504088896340736)
    AC, B_ = f32(f32(-0.5) * LOG2E), f32(-LOG2E)
    for j in range(lo, hi):
        g = int(pl[j])
        r = rec[g]
        dx, dy = f32(r[0] - f32(px)), f32(r[1] - f32(py))
        a, b, c, o = r[2], r[3], r[4], r[5]
        power = f32(f32(f32(-0.5) * f32(f32(f32(a * dx) * dx) + f32(f32(c * dy) * dy))) - f32(f32(b * dx) * dy))
        G = f32(np.exp(np.float64(power)))
        alpha = min(f32(0.99), f32(o * G))
        na, nb, nc_ = f32(AC * a), f32(B_ * b), f32(AC * c)
        lp = fma(f32(na * dx), dx, fma(f32(nc_ * dy), dy, fma(f32(nb * dx), dy, r[11])))
        af = min(f32(0.99), f32(f32(np.exp2(np.float64(lp))) * f32(1.0 / 255.0)))
        k = j - lo + 1
        hit_ref = not (power > 0) and alpha >= f32(1.0) / f32(255.0)
        test_T = f32(T * f32(1 - alpha)) if hit_ref else T
        rows.append((k, g, float(power), float(alpha), float(af), float(lp), float(r[10]), hit_ref, float(T), float(test_T)))
        if hit_ref:
            if test_T < f32(0.0001):
                rows[-1] = rows[-1] + ("SAT",)
                break
            T = test_T
    lastk = max(nc_gpu, nc_ref)
    print(f"  pixel ({px},{py}) tile {tile}: n_contrib gpu {nc_gpu} oracle {nc_ref}")
    for row in rows:
        if row[0] > lastk + 2 or (row[0] < min(nc_gpu, nc_ref) - show and not (abs(row[5]) < 10 * row[6])):
            continue
        print("   k=%d g=%d power=%.9g a_ref=%.9g a_fast=%.9g lp=%.6g eps=%.3g hit=%s T=%.9g testT=%.9g %s" %
              (row[0], row[1], row[2], row[3], row[4], row[5], row[6], row[7], row[8], row[9],
               row[10] if len(row) > 10 else ""))


def main(names):
    import test_gpu_rasterizer as tg
    from helpers import make_case
    for case in tg.CASES:
        if names and case["name"] not in names:
            continue
        cam, gs = make_case(P=case["P"], W=case["W"], H=case["H"], sh_degree=case.get("sh_degree", 0),
                            camera=case.get("camera", "identity"))
        gs = tg.mutate(gs, case.get("mutate"))
        kw = dict(mode=case["mode"], bg=case.get("bg", (0.0, 0.0, 0.0)),
                  scale_modifier=case.get("scale_modifier", 1.0), sh_degree=case.get("sh_degree", 0))
        st = tg.run_gpu(cam, gs, cov=case.get("cov", False), **kw)
        ref = tg.run_oracle(cam, gs, cov3=st["cov3"].cpu().numpy() if case.get("cov") else None, **kw)
        W, H = cam.image_width, cam.image_height
        bad = np.nonzero(st["n_contrib"] != ref["n_contrib"])[0]
        print(f"{case['name']}: {len(bad)} differing pixels", flush=True)
        gx = (W + 15) // 16
        for pix in bad[:8]:
            px, py = int(pix % W), int(pix // W)
            tile = (py // 16) * gx + px // 16
            replay(st["rec"], st["point_list"], st["ranges"], tile, px, py, int(st["n_contrib"][pix]),
                   int(ref["n_contrib"][pix]))


if __name__ == "__main__":
    main(sys.argv[1:])
