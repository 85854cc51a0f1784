#!/usr/bin/env python
"""Visible-only shade timed on a culling scene: the fused render() step
(gsr.relit.render, debug=False, fix_sky=True, bench.py's relit loss) on cfg2c's Trevi-class
cloud (1.5M Gaussians, 1920x1080, ~23 % culled) and on cfg3's cloud, with the shade deferred
into the rasterizer's forward (GSR_RELIT_VISIBLE=1: visible Gaussians only, on a second
stream beside the depth sort) against shading every Gaussian first (=0).  One stream, views
one at a time; the modes alternate over several rounds.  Prints ms per view, the shade
stages' HIP-event times and the culled fraction.  GPU box only.

    python tools/relit_visible_ab.py [rounds] [steps]
"""
import os
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd")]

import torch  # noqa: E402


def scene(name, dev):
    from gsr import scenes
    gen = torch.Generator().manual_seed(7)
    if name == "cfg2c":
        cam, gs, _ = scenes.build_config("cfg2c", device="cpu", seed=0)
        is_sky = gs["is_sky"]
    else:  # cfg3: cfg2's cloud, 1M foreground + 10 % sky (bench.py relight_leg)
        P_fg = 1_000_000
        cam, gs, _ = scenes.build_config("cfg2", device="cpu", seed=0, P=P_fg + P_fg // 10)
        is_sky = torch.zeros(gs["means3D"].shape[0], dtype=torch.bool)
        is_sky[P_fg:] = True
    P_fg = int((~is_sky).sum())
    leaves = {"xyz": gs["means3D"], "rotation": gs["rotations"], "opacity": gs["opacities"],
              "albedo": torch.rand(P_fg, 3, generator=gen), "roughness": torch.rand(P_fg, 1, generator=gen) * 0.9 + 0.05,
              "metalness": torch.rand(P_fg, 1, generator=gen)}
    leaves = {k: v.to(dev) for k, v in leaves.items()}
    base = torch.randn(25, 3, generator=gen) * 0.3
    base[0] = 1.0
    W, H = cam.image_width, cam.image_height
    view = types.SimpleNamespace(image_width=W, image_height=H, FoVx=cam.FoVx, FoVy=cam.FoVy,
                                 world_view_transform=cam.world_view_transform.to(dev),
                                 full_proj_transform=cam.full_proj_transform.to(dev),
                                 camera_center=cam.camera_center.to(dev), sky_mask=torch.ones(1, H, W, device=dev))
    names = ("render", "diffuse_color", "specular_color", "depth", "normal", "alpha", "normal_ref")
    dw = tuple(torch.randn(3, H, W, generator=gen).to(dev) for _ in names)
    return dict(leaves=leaves, scaling=gs["scales"].to(dev), is_sky=is_sky.to(dev)[:, None], base=base.to(dev),
                view=view, names=names, dw=dw)


def step(sc):
    import bench
    import relit_shade
    from gsr import relit
    t = {k: v.detach().requires_grad_(True) for k, v in sc["leaves"].items()}
    light = relit_shade.EnvironmentLight(sc["base"].clone().requires_grad_(True), sh_degree=4)
    pc = bench._RelitModel(get_xyz=t["xyz"], get_rotation=t["rotation"], get_scaling=sc["scaling"],
                           get_opacity=t["opacity"], get_is_sky=sc["is_sky"], get_albedo=t["albedo"],
                           get_roughness=t["roughness"], get_metalness=t["metalness"])
    pipe = types.SimpleNamespace(compute_cov3D_python=False)
    out = relit.render(sc["view"], pc, light, torch.zeros(1, 4, 3, device="cuda"), 1, pipe,
                       torch.zeros(3, device="cuda"), debug=False, fix_sky=True)
    loss = bench._WeightedSum.apply(sc["dw"], *[out[k] for k in sc["names"]])
    loss.backward()
    return out


def main():
    from gsr import _lib
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda")
    for name in ("cfg2c", "cfg3"):
        sc = scene(name, dev)
        out = step(sc)
        torch.cuda.synchronize()
        culled = float((out["radii"] == 0).float().mean())
        res = {"0": [], "1": [], "side": []}
        stages = {}
        for r in range(rounds):
            for mode in ("0", "1", "side"):
                os.environ["GSR_RELIT_VISIBLE"] = "0" if mode == "0" else "1"
                if mode == "side":
                    os.environ["GSR_RELIT_SIDE"] = "1"
                else:
                    os.environ.pop("GSR_RELIT_SIDE", None)
                for _ in range(3):
                    step(sc)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    step(sc)
                torch.cuda.synchronize()
                res[mode].append((time.perf_counter() - t0) * 1e3 / steps)
                if r == rounds - 1:
                    _lib.profile_read(reset=True)
                    _lib.profile_stages(["shade_fwd", "shade_bwd", "preprocess", "depth_sort", "render_fwd_mc"])
                    _lib.profile_enable(True)
                    for _ in range(5):
                        step(sc)
                    torch.cuda.synchronize()
                    _lib.profile_enable(False)
                    live = _lib.profile_read(reset=True)
                    _lib.profile_stages(None)
                    stages[mode] = {k: round(v[0] / v[1], 4) for k, v in live.items() if v[1] > 0}
        print(f"{name}: P={sc['leaves']['xyz'].shape[0]} culled {culled:.3f}", flush=True)
        for mode, lab in (("0", "shade all first       "), ("1", "visible-only, in-call "),
                          ("side", "visible-only, 2nd str.")):
            print(f"  {lab} ms/view " + " ".join(f"{x:.3f}" for x in res[mode]) + f"  stages {stages.get(mode)}",
                  flush=True)
        del sc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
