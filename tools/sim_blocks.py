#!/usr/bin/env python
"""Design simulation (CPU, C oracle): how many (Gaussian, pixel-group) evaluations would the
tile passes run with 8x8 quadrants (today) versus 4x4 blocks packed four to an evaluation
(one block per lane group of 16, the four lane groups owning the four blocks of each
quadrant's 2x2 block pattern), and how many of the evaluated lanes do useful work (alpha >=
1/255 at a pixel still blending: position < the pixel's n_contrib).

Reach per group: the exact minimum of the conic quadratic over the group's pixel box
(box_reachable without the rounding margin), and positions below the group's largest
n_contrib (the backward's limit).  cfg2 scene, 64 random tiles.

    python tools/sim_blocks.py [ntiles]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd")]


def qmin_box(a, b, c, dx0, dx1, dy0, dy1):
    inside = (dx0 <= 0) & (dx1 >= 0) & (dy0 <= 0) & (dy1 >= 0)
    q = np.full(a.shape, np.inf)
    for X in (dx0, dx1):
        y = np.clip(-b * X / c, dy0, dy1)
        q = np.minimum(q, a * X * X + 2 * b * X * y + c * y * y)
    for Y in (dy0, dy1):
        x = np.clip(-b * Y / a, dx0, dx1)
        q = np.minimum(q, a * x * x + 2 * b * x * Y + c * Y * Y)
    return np.where(inside, 0.0, q)


def main(ntiles=64):
    from oracle import oracle as orc
    from gsr import scenes
    cam, gs, c = scenes.build_config("cfg2", device="cpu", seed=0)
    W, H = cam.image_width, cam.image_height
    n = lambda t: t.numpy().astype(np.float32)
    geom = orc.preprocess(n(gs["means3D"]), n(gs["scales"]), n(gs["rotations"]), n(gs["opacities"]).reshape(-1),
                          n(gs["shs"]), None, None, n(cam.world_view_transform), n(cam.full_proj_transform),
                          n(cam.camera_center), W, H, cam.tanfovx, cam.tanfovy, 1.0, c["sh_degree"])
    R, keys, vals, ranges = orc.binning(geom, W, H)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    tiles = np.random.default_rng(5).choice(gx * gy, ntiles, replace=False).astype(np.int32)
    _, fT, nc = orc.render_fwd(ranges, vals, geom["means2D"], geom["rgb"], geom["conic_opacity"],
                               np.zeros(3, np.float32), W, H, tiles=tiles)
    nc = nc.reshape(H, W)
    tot = {"quad_evals": 0, "block_evals": 0, "useful": 0, "entries": 0, "quad_lane_evals": 0}
    for t in tiles:
        tx, ty = (t % gx) * 16, (t // gx) * 16
        lo, hi = ranges[t]
        ids = vals[lo:hi].astype(np.int64)
        pos = np.arange(hi - lo)
        mx, my = geom["means2D"][ids, 0].astype(np.float64), geom["means2D"][ids, 1].astype(np.float64)
        ca, cb, cc, op = (geom["conic_opacity"][ids, k].astype(np.float64) for k in range(4))
        thr = 2 * np.log(np.maximum(255 * op, 1e-30))
        ncp = np.zeros((16, 16), np.int64)
        hh, ww = min(16, H - ty), min(16, W - tx)
        ncp[:hh, :ww] = nc[ty:ty + hh, tx:tx + ww]
        # useful lanes: alpha >= 1/255 and position < n_contrib, per pixel
        py, px = np.mgrid[0:16, 0:16]
        useful = 0
        for k in range(len(ids)):
            dx, dy = mx[k] - (tx + px), my[k] - (ty + py)
            power = -0.5 * (ca[k] * dx * dx + cc[k] * dy * dy) - cb[k] * dx * dy
            alpha = np.minimum(0.99, op[k] * np.exp(power))
            act = (power <= 0) & (alpha >= 1 / 255) & (pos[k] < ncp) & (px < ww) & (py < hh)
            useful += int(act.sum())
        # quadrants (8x8) and blocks (4x4)
        def reach(x0, y0, s):
            lim = ncp[y0 - ty:y0 - ty + s, x0 - tx:x0 - tx + s].max()
            q = qmin_box(ca, cb, cc, x0 - mx, x0 + s - 1 - mx, y0 - my, y0 + s - 1 - my)
            return (q <= thr) & (pos < lim)
        qe = sum(reach(tx + 8 * (q & 1), ty + 8 * (q >> 1), 8).astype(int) for q in range(4))
        blk = np.stack([reach(tx + 4 * bx, ty + 4 * by, 4) for by in range(4) for bx in range(4)], 1)  # [n,16]
        # class of block (bx, by) = (bx & 1) + 2 (by & 1): one block per class per evaluation
        cls = np.array([(bx & 1) + 2 * (by & 1) for by in range(4) for bx in range(4)])
        per_cls = np.stack([blk[:, cls == k].sum(1) for k in range(4)], 1)
        be = per_cls.max(1)
        tot["quad_evals"] += int(qe.sum())
        tot["block_evals"] += int(be.sum())
        tot["useful"] += useful
        tot["entries"] += len(ids)
    T = len(tiles)
    print(f"cfg2, {T} tiles: list entries {tot['entries'] / T:.0f} per tile")
    print(f"  quadrant evaluations {tot['quad_evals'] / T:.1f} per tile, useful lanes per evaluation "
          f"{tot['useful'] / tot['quad_evals']:.1f} of 64")
    print(f"  packed 4x4-block evaluations {tot['block_evals'] / T:.1f} per tile, useful lanes per evaluation "
          f"{tot['useful'] / tot['block_evals']:.1f} of 64 ({tot['block_evals'] / tot['quad_evals']:.3f}x the evaluations)")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 64)
