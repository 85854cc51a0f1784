#!/usr/bin/env python
"""Time the rasterizer backward call (_C.rasterize_gaussians_backward) with the reference's full
output set against the autograd node's (no dL_dcolors / dL_dcov3D for an empty colors_precomp /
cov3D_precomp), alternating, on a bench configuration.  HIP events on the current stream.

    python tools/bwd_outputs_time.py [cfg2|cfg5] [iterations]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main(cfg_name="cfg2", iters=20):
    from diff_gaussian_rasterization import _C
    from gsr import scenes
    iters = int(iters)
    dev = torch.device("cuda")
    cam, gs_cpu, cfg = scenes.build_config(cfg_name, device="cpu", seed=0)
    W, H, deg = cam.image_width, cam.image_height, cfg["sh_degree"]
    g = {k: v.to(dev) for k, v in gs_cpu.items()}
    e = torch.empty(0, device=dev)
    bg = torch.zeros(3, device=dev)
    dout = torch.randn(3, H, W, generator=torch.Generator().manual_seed(1)).to(dev)
    vm, pm, cp = (cam.world_view_transform.to(dev), cam.full_proj_transform.to(dev), cam.camera_center.to(dev))
    R, color, radii, geom, binb, img = _C.rasterize_gaussians(
        bg, g["means3D"], e, g["opacities"], g["scales"], g["rotations"], 1.0, e, vm, pm, cam.tanfovx, cam.tanfovy,
        H, W, g["shs"], deg, cp, False)

    def bwd(full):
        return _C.rasterize_gaussians_backward(bg, g["means3D"], radii, e, g["scales"], g["rotations"], 1.0, e, vm,
                                               pm, cam.tanfovx, cam.tanfovy, dout, g["shs"], deg, cp, geom, R, binb,
                                               img, colors_grad=full, cov3D_grad=full)

    times = {True: [], False: []}
    for it in range(iters + 3):
        for full in (True, False):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            out = bwd(full)
            b.record()
            torch.cuda.synchronize()
            del out
            if it >= 3:
                times[full].append(a.elapsed_time(b))
    for full in (True, False):
        t = np.array(times[full])
        print(f"{cfg_name} backward call, {'full outputs (the _C contract)' if full else 'autograd (no dL_dcolors, dL_dcov3D)'}:"
              f" median {np.median(t):.4f} ms, min {t.min():.4f} over {len(t)}")


if __name__ == "__main__":
    main(*sys.argv[1:])
