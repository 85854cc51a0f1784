"""Multi-channel composite (gsr_forward_channels / gsr_backward_channels, SURVEY §8f #1's
multi-channel alternative): one composite of every channel of render()'s same-geometry
calls must equal the separate 3-channel calls -- bit for bit in the forward (the blend
decisions do not depend on the colours), and in the backward the colour gradients are the
separate calls' while the geometric gradients are their sum (float summation order
differs: relative L2 bar 1e-5)."""
import pytest
import torch

from helpers import make_case

pytestmark = pytest.mark.gpu


def _setup(P=3000, W=150, H=100, seed=0, camera="orbit"):
    import diff_gaussian_rasterization as dgr
    cam, gs = make_case(P=P, W=W, H=H, sh_degree=0, seed=seed, camera=camera)
    dev = torch.device("cuda")
    g = {k: v.to(dev) for k, v in gs.items()}
    s = dgr.GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
        bg=torch.tensor([0.1, 0.2, 0.3], device=dev), scale_modifier=1.0,
        viewmatrix=cam.world_view_transform.to(dev), projmatrix=cam.full_proj_transform.to(dev), sh_degree=-1,
        campos=cam.camera_center.to(dev), prefiltered=False)
    return dgr, g, s


def _colour_sets(P, ks, seed=3):
    gen = torch.Generator(device="cuda").manual_seed(seed)
    return [torch.rand(P, k, device="cuda", generator=gen) * 2 - 0.5 for k in ks]


def _separate(dgr, g, s, cols, bgs, weights):
    """Reference: one 3-channel call per colour set (1-channel sets padded to 3)."""
    leaves = {k: g[k].clone().requires_grad_(True) for k in ("means3D", "opacities", "scales", "rotations")}
    means2D = torch.zeros_like(leaves["means3D"], requires_grad=True)
    cl = [c.clone().requires_grad_(True) for c in cols]
    imgs, radii = [], None
    for c, bg in zip(cl, bgs):
        k = c.shape[1]
        c3 = c if k == 3 else torch.cat([c, torch.zeros(c.shape[0], 3 - k, device="cuda")], 1)
        b3 = bg if k == 3 else torch.cat([bg, torch.zeros(3 - k, device="cuda")])
        img, radii = dgr.GaussianRasterizer(s._replace(bg=b3))(
            means3D=leaves["means3D"], means2D=means2D, opacities=leaves["opacities"], colors_precomp=c3,
            scales=leaves["scales"], rotations=leaves["rotations"])
        imgs.append(img[:k])
    loss = sum((w * im).sum() for w, im in zip(weights, imgs))
    loss.backward()
    grads = [leaves[k].grad for k in ("means3D", "opacities", "scales", "rotations")] + [means2D.grad]
    return imgs, radii, grads, [c.grad for c in cl]


def _multi(dgr, g, s, cols, bgs, weights):
    leaves = {k: g[k].clone().requires_grad_(True) for k in ("means3D", "opacities", "scales", "rotations")}
    means2D = torch.zeros_like(leaves["means3D"], requires_grad=True)
    cl = [c.clone().requires_grad_(True) for c in cols]
    imgs, radii = dgr.GaussianRasterizer(s).render_channels(
        means3D=leaves["means3D"], means2D=means2D, opacities=leaves["opacities"], colors=cl, backgrounds=bgs,
        scales=leaves["scales"], rotations=leaves["rotations"])
    loss = sum((w * im).sum() for w, im in zip(weights, imgs))
    loss.backward()
    grads = [leaves[k].grad for k in ("means3D", "opacities", "scales", "rotations")] + [means2D.grad]
    return imgs, radii, grads, [c.grad for c in cl]


def _rel(a, b):
    return float(torch.linalg.norm((a - b).double()) / torch.linalg.norm(b.double()).clamp_min(1e-30))


# render()'s channel layout: image, diffuse, specular (3 each), depth (1), normal (3), alpha (1)
# = 14 channels; 22 = the debug extras too (two groups of <= 16); 1 and 5 exercise the
# narrow templates and padding.
@pytest.mark.parametrize("ks", [(3, 3, 3, 1, 3, 1), (3, 3, 3, 1, 3, 3, 1, 1, 3, 1), (1,), (3, 2), (3,)])
def test_channels_match_separate_calls(ks):
    dgr, g, s = _setup()
    P = g["means3D"].shape[0]
    cols = _colour_sets(P, ks)
    gen = torch.Generator(device="cuda").manual_seed(9)
    bgs = [torch.rand(k, device="cuda", generator=gen) for k in ks]
    weights = [torch.randn(k, s.image_height, s.image_width, device="cuda", generator=gen) for k in ks]
    imgs_s, radii_s, grads_s, cg_s = _separate(dgr, g, s, cols, bgs, weights)
    imgs_m, radii_m, grads_m, cg_m = _multi(dgr, g, s, cols, bgs, weights)
    assert torch.equal(radii_m, radii_s)
    for a, b in zip(imgs_m, imgs_s):
        assert torch.equal(a, b), float((a - b).abs().max())
    for a, b in zip(cg_m, cg_s):
        assert _rel(a, b) < 1e-5
    for name, a, b in zip(("means3D", "opacities", "scales", "rotations", "means2D"), grads_m, grads_s):
        assert _rel(a, b) < 1e-5, (name, _rel(a, b))


@pytest.mark.parametrize("ks", [(3, 3, 3, 1, 3, 1), (3, 2)])
def test_channels_match_separate_calls_exact(ks):
    """Exact blend mode (gsr_set_exact_blend) in both: the composite's channels equal the separate
    exact-mode 3-channel calls bit for bit (their blend arithmetic is the same expression per
    channel), the gradients as in the default mode."""
    from gsr import _lib
    with _lib.exact_blend_mode():
        test_channels_match_separate_calls(ks)


def test_channels_heavy_tiles_and_ragged():
    """Dense centre (heavy-tile quadrant split) on a ragged image size."""
    dgr, g, s = _setup(P=40000, W=133, H=77, seed=5, camera="identity")
    P = g["means3D"].shape[0]
    ks = (3, 3, 1)
    cols = _colour_sets(P, ks, seed=4)
    bgs = [torch.zeros(k, device="cuda") for k in ks]
    gen = torch.Generator(device="cuda").manual_seed(2)
    weights = [torch.randn(k, s.image_height, s.image_width, device="cuda", generator=gen) for k in ks]
    imgs_s, _, grads_s, cg_s = _separate(dgr, g, s, cols, bgs, weights)
    imgs_m, _, grads_m, cg_m = _multi(dgr, g, s, cols, bgs, weights)
    for a, b in zip(imgs_m, imgs_s):
        assert torch.equal(a, b)
    for a, b in zip(cg_m + grads_m, cg_s + grads_s):
        assert _rel(a, b) < 1e-5


def test_channels_empty_and_culled():
    import diff_gaussian_rasterization as dgr
    _, g, s = _setup(P=500)
    r = dgr.GaussianRasterizer(s)
    e = torch.zeros(0, 3, device="cuda")
    imgs, radii = r.render_channels(means3D=e, means2D=e.clone(), opacities=torch.zeros(0, 1, device="cuda"),
                                    colors=[torch.zeros(0, 2, device="cuda")], scales=e.clone(),
                                    rotations=torch.zeros(0, 4, device="cuda"))
    assert imgs[0].shape == (2, s.image_height, s.image_width) and radii.numel() == 0
    # everything behind the camera: background everywhere
    m = g["means3D"].clone()
    m[:, 2] = -5.0
    bg = torch.tensor([0.25, 0.5, 0.75, 1.0], device="cuda")
    imgs, radii = r.render_channels(means3D=m, means2D=torch.zeros_like(m), opacities=g["opacities"],
                                    colors=[torch.rand(m.shape[0], 4, device="cuda")], backgrounds=[bg],
                                    scales=g["scales"], rotations=g["rotations"])
    assert int((radii > 0).sum()) == 0
    assert torch.equal(imgs[0], bg.view(4, 1, 1).expand(4, s.image_height, s.image_width))


def test_channels_bad_arguments():
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import _C
    _, g, s = _setup(P=100)
    with pytest.raises(ValueError):
        _C.rasterize_gaussians_channels(torch.zeros(2, device="cuda"), g["means3D"],
                                        torch.zeros(100, 3, device="cuda"), g["opacities"], g["scales"],
                                        g["rotations"], 1.0, torch.Tensor([]), s.viewmatrix, s.projmatrix, s.tanfovx,
                                        s.tanfovy, s.image_height, s.image_width, s.campos, False)
    with pytest.raises(Exception):
        dgr.GaussianRasterizer(s).render_channels(means3D=g["means3D"], means2D=g["means3D"],
                                                  opacities=g["opacities"], colors=[g["means3D"]])


@pytest.mark.parametrize("W,H", [(640, 360), (8320, 40), (40, 8320)], ids=["640x360", "wide_520_tiles", "tall_520_rows"])
def test_channels_frame_shapes(W, H):
    """render()'s 14-channel layout on a frame with cost-balanced backward bands (640x360) and on
    strips of more than 512 tiles per row / tile rows, where the bands fall back to equal tile
    counts (gsr_order.hpp balanced_band)."""
    dgr, g, s = _setup(P=6000, W=W, H=H, seed=7, camera="identity")
    P = g["means3D"].shape[0]
    ks = (3, 3, 3, 1, 3, 1)
    cols = _colour_sets(P, ks, seed=6)
    gen = torch.Generator(device="cuda").manual_seed(8)
    bgs = [torch.rand(k, device="cuda", generator=gen) for k in ks]
    weights = [torch.randn(k, H, W, device="cuda", generator=gen) for k in ks]
    imgs_s, radii_s, grads_s, cg_s = _separate(dgr, g, s, cols, bgs, weights)
    imgs_m, radii_m, grads_m, cg_m = _multi(dgr, g, s, cols, bgs, weights)
    assert torch.equal(radii_m, radii_s)
    for a, b in zip(imgs_m, imgs_s):
        assert torch.equal(a, b)
    for a, b in zip(cg_m + grads_m, cg_s + grads_s):
        assert _rel(a, b) < 1e-5
