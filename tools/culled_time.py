#!/usr/bin/env python
"""cfg2's cloud with a share of the Gaussians pushed out of the frustum at random (the
interleaved-culling case of real views; tests/test_gpu_rasterizer.py's 'shift' edge case at
scale), one forward + backward per step through the drop-in _C: for a rocprofv3 kernel trace
of the preprocess passes (tools only; GPU box).

    python tools/culled_time.py [fraction_culled] [steps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd")]

import torch  # noqa: E402


def main():
    from diff_gaussian_rasterization import _C
    from gsr import scenes
    frac = float(sys.argv[1]) if len(sys.argv) > 1 else 0.5
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    cam, gs, cfg = scenes.build_config("cfg2", device="cpu", seed=0)
    g = torch.Generator().manual_seed(3)
    out = torch.rand(gs["means3D"].shape[0], generator=g) < frac
    gs["means3D"][out, 0] += 4.0 * gs["means3D"][out, 2]  # far right of the frustum: zero-area rects
    d = {k: v.to(dev) for k, v in gs.items()}
    W, H, deg = cam.image_width, cam.image_height, cfg["sh_degree"]
    e = torch.empty(0, device=dev)
    bg = torch.zeros(3, device=dev)
    dout = torch.randn(3, H, W, device=dev)
    c = cam.to(dev)
    vm, pm, cp = c.world_view_transform, c.full_proj_transform, c.camera_center

    def step():
        R, color, radii, geom, binb, img = _C.rasterize_gaussians(bg, d["means3D"], e, d["opacities"], d["scales"],
                                                                  d["rotations"], 1.0, e, vm, pm, cam.tanfovx,
                                                                  cam.tanfovy, H, W, d["shs"], deg, cp, False)
        _C.rasterize_gaussians_backward(bg, d["means3D"], radii, e, d["scales"], d["rotations"], 1.0, e, vm, pm,
                                        cam.tanfovx, cam.tanfovy, dout, d["shs"], deg, cp, geom, R, binb, img)
        return radii

    for _ in range(3):
        radii = step()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(steps):
        step()
    ev[1].record()
    torch.cuda.synchronize()
    print(f"visible {int((radii > 0).sum())} of {radii.numel()}: {ev[0].elapsed_time(ev[1]) / steps:.4f} ms per call pair")


if __name__ == "__main__":
    main()
