#!/usr/bin/env python
"""Per-tile list-length and n_contrib distribution of one forward call (load-balance view)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd"), os.path.join(ROOT, "tests")]


def main(src="cfg2"):
    from gsr import scenes
    from test_gpu_rasterizer import run_gpu
    if src.endswith(".ply"):
        cam, gs, c = scenes.ply_config(src)
    else:
        cam, gs, c = scenes.build_config(src)
    st = run_gpu(cam, gs, mode="sh", sh_degree=c["sh_degree"])
    rg = st["ranges"].astype(np.int64)
    n = rg[:, 1] - rg[:, 0]
    W, H = cam.image_width, cam.image_height
    nc = st["n_contrib"].reshape(H, W)
    q = lambda a, p: int(np.percentile(a, p))
    print(f"{src}: R={st['R']} tiles={len(n)} nonempty={(n > 0).sum()} list len p50={q(n, 50)} p99={q(n, 99)} "
          f"max={n.max()} | n_contrib p50={q(nc, 50)} p99={q(nc, 99)} max={nc.max()}")


if __name__ == "__main__":
    main(*sys.argv[1:])
