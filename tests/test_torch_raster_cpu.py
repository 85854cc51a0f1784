"""The PyTorch-CPU baseline rasterizer (oracle/torch_raster.py, timed by bench.py's
cpu_baseline) against the C oracle on the same inputs: per-Gaussian screen geometry,
binning, images and all gradients.  Not bit-exact (PyTorch's op order and vectorised
arithmetic), so float bars."""
import numpy as np
import pytest
import torch

from helpers import make_case, np32, rel_l2
from oracle import oracle as orc
from oracle import torch_raster as tr


@pytest.mark.parametrize("deg,camera,W,H", [(0, "identity", 64, 48), (3, "orbit", 70, 45)])
def test_torch_rasterizer_matches_oracle(deg, camera, W, H):
    cam, gs = make_case(P=1500, W=W, H=H, sh_degree=deg, camera=camera)
    vm, pm, cp = cam.world_view_transform, cam.full_proj_transform, cam.camera_center
    bg = torch.tensor([0.1, 0.2, 0.3])
    leaves = [gs["means3D"].clone().requires_grad_(True), gs["scales"].clone().requires_grad_(True),
              gs["rotations"].clone().requires_grad_(True), gs["shs"].clone().requires_grad_(True)]
    pre = tr.preprocess(leaves[0], leaves[1], leaves[2], gs["opacities"], leaves[3], deg, vm, pm, cp, W, H,
                        cam.tanfovx, cam.tanfovy)
    ref = orc.forward(np32(bg), np32(gs["means3D"]), None, np32(gs["opacities"]), np32(gs["scales"]),
                      np32(gs["rotations"]), 1.0, None, np32(vm), np32(pm), cam.tanfovx, cam.tanfovy, H, W,
                      np32(gs["shs"]), deg, np32(cp))
    radii = pre["radii"].numpy()
    assert (radii == ref["radii"]).mean() > 0.995
    vis = (radii > 0) & (ref["radii"] > 0)
    np.testing.assert_allclose(pre["xy"].numpy()[vis], ref["means2D"][vis], rtol=1e-5, atol=1e-3)
    assert rel_l2(pre["conic"].detach().numpy()[vis], ref["conic_opacity"][vis, :3]) < 1e-4
    pl, ranges = tr.binning(pre, W, H)
    if (radii == ref["radii"]).all():
        np.testing.assert_array_equal(pl.numpy(), ref["point_list"].astype(np.int64))
    T = ranges.shape[0]
    tiles = torch.arange(T)
    color, fT, nc, inside, = tr.render_fwd(tiles, ranges, pl, pre["xy"], pre["conic"].detach(), pre["opacity"],
                                          pre["rgb"].detach(), bg, W, H)
    img = tr.to_image(color, tiles, W, H)
    assert rel_l2(img.numpy(), ref["color"]) < 1e-4
    dout = torch.randn(3, H, W, generator=torch.Generator().manual_seed(3))
    rb = tr.render_bwd(1500, tiles, ranges, pl, pre["xy"], pre["conic"].detach(), pre["opacity"],
                       pre["rgb"].detach(), bg, fT, nc, tr.from_image(dout, tiles, W, H), W, H)
    grads = tr.preprocess_bwd(pre, leaves, rb["dL_dmean2D"], rb["dL_dconic"], rb["dL_dcolors"])
    gref = orc.backward(ref, np32(bg), np32(gs["means3D"]), None, np32(gs["scales"]), np32(gs["rotations"]), 1.0,
                        None, np32(vm), np32(pm), cam.tanfovx, cam.tanfovy, dout.numpy(), np32(gs["shs"]), deg,
                        np32(cp))
    for name, mine in (("dL_dmean2D", rb["dL_dmean2D"]), ("dL_dopacity", rb["dL_dopacity"]),
                       ("dL_dconic", rb["dL_dconic"]), ("dL_dmeans3D", grads[0]), ("dL_dscales", grads[1]),
                       ("dL_drotations", grads[2]), ("dL_dsh", grads[3])):
        r = gref[name]
        e = rel_l2(mine.detach().numpy().reshape(r.shape), r)
        assert e < 1e-4, (name, e)
