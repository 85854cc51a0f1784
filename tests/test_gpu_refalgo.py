"""The reference-structure GPU baseline (baseline/refalgo.hip) computes the reference's
images and gradients: parity with the CPU oracle on the rasterizer cases, and with libgsr
at cfg2 size.  bench.py divides by its time, so it has to be a correct rasterizer."""
import numpy as np
import pytest
import torch

from helpers import make_case, np32, rel_l2
from oracle import oracle as orc
from test_gpu_rasterizer import mutate

pytestmark = pytest.mark.gpu

TOL = 1e-4
CASES = [
    dict(name="sh0", P=3000, W=128, H=128, mode="sh", sh_degree=0),
    dict(name="colors_ragged_bg", P=2500, W=100, H=75, mode="colors", bg=(0.2, 0.5, 1.0)),
    dict(name="sh3_orbit", P=2500, W=96, H=64, mode="sh", sh_degree=3, camera="orbit"),
    dict(name="opaque_stack", P=6000, W=64, H=64, mode="sh", sh_degree=1, mutate="opaque"),
    dict(name="heavy_tiles", P=70000, W=64, H=48, mode="colors", mutate="thin"),
]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_refalgo_matches_oracle(case):
    from baseline.refalgo import RefAlgoRasterizer
    cam, gs = make_case(P=case["P"], W=case["W"], H=case["H"], sh_degree=case.get("sh_degree", 0),
                        camera=case.get("camera", "identity"))
    gs = mutate(gs, case.get("mutate"))
    W, H, deg = cam.image_width, cam.image_height, case.get("sh_degree", 0)
    bg = np.asarray(case.get("bg", (0.0, 0.0, 0.0)), np.float32)
    dev = torch.device("cuda")
    e = torch.empty(0, device=dev)
    colors = gs["colors"].to(dev) if case["mode"] == "colors" else e
    sh = gs["shs"].to(dev) if case["mode"] == "sh" else e
    g = {k: v.to(dev) for k, v in gs.items()}
    vm, pm, cp = cam.world_view_transform.to(dev), cam.full_proj_transform.to(dev), cam.camera_center.to(dev)
    bg_t = torch.tensor(bg, device=dev)
    ras = RefAlgoRasterizer()
    R, color, radii = ras.forward(bg_t, g["means3D"], colors, g["opacities"], g["scales"], g["rotations"], 1.0, e, vm,
                                  pm, cam.tanfovx, cam.tanfovy, H, W, sh, deg, cp)
    dout = torch.randn(3, H, W, generator=torch.Generator().manual_seed(1))
    grads = ras.backward(bg_t, g["means3D"], radii, g["scales"], g["rotations"], 1.0, e, vm, pm, cam.tanfovx,
                         cam.tanfovy, dout.to(dev), sh, deg, cp)
    torch.cuda.synchronize()
    ref = orc.forward(bg, np32(gs["means3D"]), np32(gs["colors"]) if case["mode"] == "colors" else None,
                      np32(gs["opacities"]), np32(gs["scales"]), np32(gs["rotations"]), 1.0, None,
                      np32(cam.world_view_transform), np32(cam.full_proj_transform), cam.tanfovx, cam.tanfovy, H, W,
                      np32(gs["shs"]) if case["mode"] == "sh" else None, deg, np32(cam.camera_center))
    assert R == ref["num_rendered"]
    np.testing.assert_array_equal(radii.cpu().numpy(), ref["radii"])
    assert rel_l2(color.cpu().numpy(), ref["color"]) <= TOL
    gref = orc.backward(ref, bg, np32(gs["means3D"]), np32(gs["colors"]) if case["mode"] == "colors" else None,
                        np32(gs["scales"]), np32(gs["rotations"]), 1.0, None, np32(cam.world_view_transform),
                        np32(cam.full_proj_transform), cam.tanfovx, cam.tanfovy, dout.numpy(),
                        np32(gs["shs"]) if case["mode"] == "sh" else None, deg, np32(cam.camera_center))
    names = ["dL_dmean2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
             "dL_drotations"]
    errs = {}
    for n, t in zip(names, grads):
        r = gref[n]
        if r.size == 0 or np.abs(r).max() == 0:
            continue
        errs[n] = rel_l2(t.cpu().numpy().reshape(r.shape), r)
    assert all(v <= TOL for v in errs.values()), errs


def test_refalgo_matches_libgsr_cfg2():
    """At BASELINE.json's full size the baseline and the product render the same image and
    the same gradients (different summation orders: relative L2)."""
    from baseline.refalgo import RefAlgoRasterizer
    from diff_gaussian_rasterization import _C
    from gsr import scenes
    cam, gs, cfg = scenes.build_config("cfg2", device="cpu", seed=0)
    dev = torch.device("cuda")
    g = {k: v.to(dev) for k, v in gs.items()}
    e = torch.empty(0, device=dev)
    bg = torch.zeros(3, device=dev)
    W, H, deg = cam.image_width, cam.image_height, cfg["sh_degree"]
    vm, pm, cp = cam.world_view_transform.to(dev), cam.full_proj_transform.to(dev), cam.camera_center.to(dev)
    dout = torch.randn(3, H, W, generator=torch.Generator().manual_seed(1)).to(dev)
    ras = RefAlgoRasterizer()
    R0, c0, r0 = ras.forward(bg, g["means3D"], e, g["opacities"], g["scales"], g["rotations"], 1.0, e, vm, pm,
                             cam.tanfovx, cam.tanfovy, H, W, g["shs"], deg, cp)
    g0 = ras.backward(bg, g["means3D"], r0, g["scales"], g["rotations"], 1.0, e, vm, pm, cam.tanfovx, cam.tanfovy,
                      dout, g["shs"], deg, cp)
    R1, c1, r1, geom, binb, img = _C.rasterize_gaussians(bg, g["means3D"], e, g["opacities"], g["scales"],
                                                         g["rotations"], 1.0, e, vm, pm, cam.tanfovx, cam.tanfovy, H,
                                                         W, g["shs"], deg, cp, False)
    g1 = _C.rasterize_gaussians_backward(bg, g["means3D"], r1, e, g["scales"], g["rotations"], 1.0, e, vm, pm,
                                         cam.tanfovx, cam.tanfovy, dout, g["shs"], deg, cp, geom, R1, binb, img)
    torch.cuda.synchronize()
    assert R0 == R1
    assert torch.equal(r0, r1)
    assert rel_l2(c0.cpu().numpy(), c1.cpu().numpy()) <= TOL
    for a, b in zip(g0, g1):
        if b.numel() and b.abs().max() > 0:
            assert rel_l2(a.cpu().numpy(), b.cpu().numpy()) <= TOL
