"""Experiment (tools only): cfg2 rasterizer fwd+bwd per view with views alternating over S
HIP streams (independent views of one mini-batch in flight together) vs one stream."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd")]
import torch  # noqa: E402

from diff_gaussian_rasterization import _C  # noqa: E402
from gsr import scenes  # noqa: E402

dev = torch.device("cuda")
cam, gs, cfg = scenes.build_config("cfg2", device="cpu", seed=0)
W, H, deg = cam.image_width, cam.image_height, cfg["sh_degree"]
g = {k: v.to(dev) for k, v in gs.items()}
e = torch.empty(0, device=dev)
bg = torch.zeros(3, device=dev)
vm, pm, cp = cam.world_view_transform.to(dev), cam.full_proj_transform.to(dev), cam.camera_center.to(dev)
dout = torch.randn(3, H, W, generator=torch.Generator().manual_seed(1)).to(dev)


def view():
    R, color, radii, geom, binb, img = _C.rasterize_gaussians(bg, g["means3D"], e, g["opacities"], g["scales"],
                                                             g["rotations"], 1.0, e, vm, pm, cam.tanfovx, cam.tanfovy,
                                                             H, W, g["shs"], deg, cp, False)
    _C.rasterize_gaussians_backward(bg, g["means3D"], radii, e, g["scales"], g["rotations"], 1.0, e, vm, pm,
                                    cam.tanfovx, cam.tanfovy, dout, g["shs"], deg, cp, geom, R, binb, img)


for ns in (1, 2, 3):
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(ns - 1)]
    for rep in range(2):
        torch.cuda.synchronize()
        n = 40
        t0 = time.perf_counter()
        for i in range(n):
            with torch.cuda.stream(streams[i % ns]):
                view()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / n
    print(f"streams {ns}: {ms:.4f} ms per view, {W * H / ms / 1e3:.1f} MPix/s", flush=True)
