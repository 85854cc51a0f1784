"""GPU parity: libgsr.so (through the C ABI via diff_gaussian_rasterization._C) vs the CPU
oracle on the same seeded inputs.

Bar (BASELINE.json north_star): bit-exact on tile/key indexing -- radii, tiles_touched,
screen means, conics, depth keys, num_rendered, the sorted instance list and the tile
ranges -- plus identical per-pixel n_contrib (every blend decision), RGB within 1e-6
absolute of the oracle per value, and within 1e-4 relative on every gradient (relative L2
over the tensor: the GPU sums gradients in a different order than the reference's
atomics, so elementwise bits cannot match; the tolerance is tied to the tensor norm)."""
import math

import numpy as np
import pytest
import torch

from helpers import make_case, np32, rel_l2
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

RGB_TOL = 1e-4
GRAD_TOL = 1e-4


def _dgr():
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import _C
    from gsr import _lib
    return dgr, _C, _lib


def _view(buf, off, n, dtype):
    base = buf.data_ptr()
    shift = (-base) % 256
    nbytes = n * torch.empty(0, dtype=dtype).element_size()
    return buf[shift + off: shift + off + nbytes].view(dtype)


def run_gpu(cam, gs, mode="colors", bg=(0.0, 0.0, 0.0), scale_modifier=1.0, sh_degree=0, prefiltered=False,
            cov=False):
    _, _C, _lib = _dgr()
    dev = torch.device("cuda")
    P = gs["means3D"].shape[0]
    W, H = cam.image_width, cam.image_height
    e = torch.empty(0, device=dev)
    means = gs["means3D"].to(dev)
    colors = gs["colors"].to(dev) if mode == "colors" else e
    sh = gs["shs"].to(dev) if mode == "sh" else e
    if cov:
        cov3 = torch.tensor(orc.preprocess(np32(gs["means3D"]), np32(gs["scales"]), np32(gs["rotations"]),
                                           np32(gs["opacities"]).reshape(-1), None, np.zeros((P, 3), np.float32),
                                           None, np.eye(4, dtype=np.float32), np.eye(4, dtype=np.float32),
                                           np.zeros(3, np.float32), 16, 16, 1.0, 1.0, scale_modifier)["cov3D"],
                            device=dev)
        scales, rots = e, e
    else:
        cov3 = e
        scales, rots = gs["scales"].to(dev), gs["rotations"].to(dev)
    bg_t = torch.tensor(bg, dtype=torch.float32, device=dev)
    vm, pm, cp = cam.world_view_transform.to(dev), cam.full_proj_transform.to(dev), cam.camera_center.to(dev)
    R, color, radii, geom, binb, img = _C.rasterize_gaussians(
        bg_t, means, colors, gs["opacities"].to(dev), scales, rots, scale_modifier, cov3, vm, pm, cam.tanfovx,
        cam.tanfovy, H, W, sh, sh_degree, cp, prefiltered)
    torch.cuda.synchronize()
    L = _lib.layout(P, R, W, H)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    st = dict(R=R, color=color, radii=radii, geom=geom, binb=binb, img=img, bg=bg_t, means=means, colors=colors,
              sh=sh, scales=scales, rots=rots, cov3=cov3, vm=vm, pm=pm, cp=cp)
    st["rec"] = _view(geom, L.geom_rec, 12 * P, torch.float32).view(P, 12).cpu().numpy()
    st["tiles"] = _view(geom, L.geom_tiles, P, torch.int32).cpu().numpy().view(np.uint32)
    st["depth_key"] = _view(geom, L.geom_depth_key, P, torch.int32).cpu().numpy().view(np.uint32)
    # the reference's point_list and tile ranges, written from the super-tile lists the
    # binning leaves (the tile passes read those directly)
    pl, rg = _lib.materialize_lists(R, W, H, binb)
    st["point_list"] = pl.cpu().numpy().view(np.uint32)
    st["ranges"] = rg.cpu().numpy().view(np.uint32).reshape(-1, 2)
    st["final_T"] = _view(img, L.img_final_T, W * H, torch.float32).cpu().numpy()
    st["n_contrib"] = _view(img, L.img_n_contrib, W * H, torch.int32).cpu().numpy().view(np.uint32)
    return st


def run_oracle(cam, gs, mode="colors", bg=(0.0, 0.0, 0.0), scale_modifier=1.0, sh_degree=0, cov3=None):
    W, H = cam.image_width, cam.image_height
    return orc.forward(np.asarray(bg, np.float32), np32(gs["means3D"]), np32(gs["colors"]) if mode == "colors" else None,
                       np32(gs["opacities"]), None if cov3 is not None else np32(gs["scales"]),
                       None if cov3 is not None else np32(gs["rotations"]), scale_modifier, cov3,
                       np32(cam.world_view_transform), np32(cam.full_proj_transform), cam.tanfovx, cam.tanfovy, H, W,
                       np32(gs["shs"]) if mode == "sh" else None, sh_degree, np32(cam.camera_center))


def check_forward(st, ref, W, H):
    vis = ref["radii"] > 0
    np.testing.assert_array_equal(st["radii"].cpu().numpy(), ref["radii"])
    np.testing.assert_array_equal(st["tiles"], ref["tiles_touched"])
    rec = st["rec"]
    # bit-exact screen-space geometry of every visible Gaussian
    np.testing.assert_array_equal(rec[vis, 0:2], ref["means2D"][vis])
    np.testing.assert_array_equal(rec[vis, 2:4], ref["conic_opacity"][vis, 0:2])
    np.testing.assert_array_equal(rec[vis, 4:6], ref["conic_opacity"][vis, 2:4])
    np.testing.assert_array_equal(rec[vis, 6:9], ref["features"][vis])
    np.testing.assert_array_equal(st["depth_key"][vis], ref["depths"][vis].view(np.uint32))
    assert st["R"] == ref["num_rendered"]
    np.testing.assert_array_equal(st["point_list"], ref["point_list"])
    np.testing.assert_array_equal(st["ranges"], ref["ranges"])
    color = st["color"].cpu().numpy()
    e = rel_l2(color, ref["color"])
    assert e <= RGB_TOL, f"rgb rel L2 {e:.3e}"
    # Measured on every case (tools/parity_margins.py, profiles/r2_parity_margins.log): no
    # blend decision differs from the oracle's expf (n_contrib identical everywhere) and no
    # value differs by more than 3e-7.  The bars are those maxima with a small margin.
    np.testing.assert_array_equal(st["n_contrib"], ref["n_contrib"])
    scale = max(1.0, float(np.abs(ref["color"]).max()))
    assert np.abs(color - ref["color"]).max() <= 1e-6 * scale, np.abs(color - ref["color"]).max()
    assert np.abs(st["final_T"] - ref["final_T"]).max() <= 1e-6
    return e


CASES = [
    dict(name="cfg1_small_sh0", P=3000, W=128, H=128, mode="sh", sh_degree=0),
    dict(name="colors_ragged", P=2500, W=100, H=75, mode="colors"),
    dict(name="sh3_orbit_bg", P=2500, W=96, H=64, mode="sh", sh_degree=3, camera="orbit", bg=(0.2, 0.5, 1.0)),
    dict(name="sh1_scale_mod", P=2000, W=64, H=64, mode="sh", sh_degree=1, scale_modifier=1.7),
    dict(name="sh2_cov_precomp", P=2000, W=80, H=48, mode="sh", sh_degree=2, cov=True),
    dict(name="dense_small", P=20000, W=64, H=64, mode="colors"),
    # edge cases: sub-tile image, Gaussians larger than the image, near-threshold and opaque
    # opacities (early saturation), a cloud half outside the frustum, SH degree 3 + colours
    dict(name="tiny_7x5", P=400, W=7, H=5, mode="colors"),
    dict(name="huge_gaussians", P=300, W=96, H=80, mode="colors", mutate="huge"),
    dict(name="faint_opacity", P=3000, W=80, H=64, mode="colors", mutate="faint"),
    dict(name="opaque_stack", P=6000, W=64, H=64, mode="sh", sh_degree=1, mutate="opaque"),
    dict(name="half_outside", P=3000, W=96, H=96, mode="sh", sh_degree=3, mutate="shift"),
    # lists above the heavy-tile thresholds (>= 8192 entries, n_contrib >= 2048): the
    # four-way quadrant split of the tile passes
    dict(name="heavy_tiles", P=70000, W=64, H=48, mode="colors", mutate="thin"),
    # depths over 12 and 20 octaves (same screen footprints): every byte of the depth keys varies
    dict(name="depth_12_octaves", P=4000, W=96, H=64, mode="colors", mutate="deep12"),
    dict(name="depth_20_octaves", P=4000, W=96, H=64, mode="sh", sh_degree=1, mutate="deep20"),
    # runs of equal depth keys across many 2048-key sort tiles and chains: the sort's stability
    # (the reference's (depth, index) order) is all that orders them
    dict(name="depth_ties", P=40000, W=96, H=64, mode="colors", mutate="ties"),
    # more than 512 tiles per row / tile rows: the backward's cost-balanced bands fall back to
    # equal bands (balanced_band scans one row or one row's tiles per thread of a 512-thread
    # workgroup)
    dict(name="wide_strip_520_tiles", P=3000, W=8320, H=40, mode="colors"),
    dict(name="tall_strip_520_rows", P=3000, W=40, H=8320, mode="sh", sh_degree=1),
]


def mutate(gs, how):
    """Edge-case variants of a synthetic cloud (deterministic)."""
    if how is None:
        return gs
    gs = {k: v.clone() for k, v in gs.items()}
    g = torch.Generator().manual_seed(11)
    if how == "huge":  # screen radii beyond the image: rects clamp to the grid, R ~ P * T
        gs["scales"] *= 25.0
    elif how == "faint":  # opacities straddling 1/255: alpha-threshold decisions everywhere
        gs["opacities"] = torch.empty_like(gs["opacities"]).uniform_(0.5 / 255, 3.0 / 255, generator=g)
    elif how == "opaque":  # opaque and large: most pixels saturate (T < 1e-4) early
        gs["opacities"].fill_(0.99)
        gs["scales"] *= 3.0
    elif how == "thin":  # low opacity, wide: long lists that never saturate
        gs["opacities"] = torch.empty_like(gs["opacities"]).uniform_(0.01, 0.03, generator=g)
        gs["scales"] *= 2.0
    elif how in ("deep12", "deep20"):  # every Gaussian pushed along its ray by 2^U(0, n)
        k = torch.pow(2.0, torch.rand(gs["means3D"].shape[0], 1, generator=g) * float(how[4:]))
        gs["means3D"] *= k
        gs["scales"] *= k
    elif how == "ties":  # every depth on a 1/4 grid: thousands of Gaussians per depth key
        gs["means3D"][:, 2] = torch.round(gs["means3D"][:, 2] * 4.0) / 4.0
    elif how == "shift":  # half the cloud left of the frustum, some behind the near plane
        gs["means3D"][:, 0] -= 0.6 * gs["means3D"][:, 2]
        gs["means3D"][: gs["means3D"].shape[0] // 10, 2] = 0.1
    return gs


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_forward_parity(case):
    cam, gs = make_case(P=case["P"], W=case["W"], H=case["H"], sh_degree=case.get("sh_degree", 0),
                        camera=case.get("camera", "identity"))
    gs = mutate(gs, case.get("mutate"))
    kw = dict(mode=case["mode"], bg=case.get("bg", (0.0, 0.0, 0.0)), scale_modifier=case.get("scale_modifier", 1.0),
              sh_degree=case.get("sh_degree", 0))
    st = run_gpu(cam, gs, cov=case.get("cov", False), **kw)
    ref = run_oracle(cam, gs, cov3=st["cov3"].cpu().numpy() if case.get("cov") else None, **kw)
    check_forward(st, ref, cam.image_width, cam.image_height)


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_forward_parity_exact(case):
    """Exact blend mode (gsr_set_exact_blend; gsr_tile.hpp "exact mode"): the forward's colours,
    final transmittance and n_contrib equal the canonical oracle's bit for bit, on every case."""
    from gsr import _lib
    cam, gs = make_case(P=case["P"], W=case["W"], H=case["H"], sh_degree=case.get("sh_degree", 0),
                        camera=case.get("camera", "identity"))
    gs = mutate(gs, case.get("mutate"))
    kw = dict(mode=case["mode"], bg=case.get("bg", (0.0, 0.0, 0.0)), scale_modifier=case.get("scale_modifier", 1.0),
              sh_degree=case.get("sh_degree", 0))
    with _lib.exact_blend_mode():
        st = run_gpu(cam, gs, cov=case.get("cov", False), **kw)
    ref = run_oracle(cam, gs, cov3=st["cov3"].cpu().numpy() if case.get("cov") else None, **kw)
    check_forward(st, ref, cam.image_width, cam.image_height)
    np.testing.assert_array_equal(st["color"].cpu().numpy(), ref["color"])
    np.testing.assert_array_equal(st["final_T"], ref["final_T"])


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_backward_parity(case):
    _, _C, _ = _dgr()
    cam, gs = make_case(P=case["P"], W=case["W"], H=case["H"], sh_degree=case.get("sh_degree", 0),
                        camera=case.get("camera", "identity"))
    gs = mutate(gs, case.get("mutate"))
    kw = dict(mode=case["mode"], bg=case.get("bg", (0.0, 0.0, 0.0)), scale_modifier=case.get("scale_modifier", 1.0),
              sh_degree=case.get("sh_degree", 0))
    st = run_gpu(cam, gs, cov=case.get("cov", False), **kw)
    cov3 = st["cov3"].cpu().numpy() if case.get("cov") else None
    ref = run_oracle(cam, gs, cov3=cov3, **kw)
    W, H = cam.image_width, cam.image_height
    g = torch.Generator().manual_seed(1)
    dout = torch.randn(3, H, W, generator=g)
    grads = _C.rasterize_gaussians_backward(
        st["bg"], st["means"], st["radii"], st["colors"], st["scales"], st["rots"], kw["scale_modifier"], st["cov3"],
        st["vm"], st["pm"], cam.tanfovx, cam.tanfovy, dout.cuda(), st["sh"], kw["sh_degree"], st["cp"], st["geom"],
        st["R"], st["binb"], st["img"])
    names = ["dL_dmean2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
             "dL_drotations"]
    gref = orc.backward(ref, np.asarray(kw["bg"], np.float32), np32(gs["means3D"]),
                        np32(gs["colors"]) if kw["mode"] == "colors" else None,
                        None if cov3 is not None else np32(gs["scales"]),
                        None if cov3 is not None else np32(gs["rotations"]), kw["scale_modifier"], cov3,
                        np32(cam.world_view_transform), np32(cam.full_proj_transform), cam.tanfovx, cam.tanfovy,
                        dout.numpy(), np32(gs["shs"]) if kw["mode"] == "sh" else None, kw["sh_degree"],
                        np32(cam.camera_center))
    errs = {}
    for n, gt in zip(names, grads):
        r = gref[n]
        if n == "dL_dcolors" and kw["mode"] == "sh":
            pass  # still returned by the reference (grad w.r.t. the absent colors_precomp)
        mine = gt.detach().cpu().numpy().reshape(r.shape)
        if r.size == 0:
            continue
        if n in ("dL_dscales", "dL_drotations") and cov3 is not None:
            assert np.abs(mine).max() == 0.0
            continue
        if n == "dL_dcov3D" and cov3 is None:
            pass
        if np.abs(r).max() == 0:
            assert np.abs(mine).max() == 0.0, n
            continue
        errs[n] = rel_l2(mine, r)
    bad = {k: v for k, v in errs.items() if v > GRAD_TOL}
    assert not bad, f"gradient rel L2 errors above {GRAD_TOL}: {bad} (all: {errs})"


@pytest.mark.parametrize("name,bits", [("heavy_tiles", 8), ("dense_small", 6), ("sh3_orbit_bg", 5)])
def test_backward_parity_quadrant_units(name, bits):
    """The backward's quadrant units: its split threshold lowered (gsr_set_backward_heavy_bits)
    so that the parity cases' tiles -- below the default 2^13 evaluations -- run as four
    quadrant units each, against the same oracle and tolerance as test_backward_parity."""
    _, _, _lib = _dgr()
    case = next(c for c in CASES if c["name"] == name)
    _lib.set_backward_heavy_bits(bits)
    try:
        test_backward_parity(case)
    finally:
        _lib.set_backward_heavy_bits(-1)


@pytest.mark.parametrize("name", ["faint_opacity", "sh3_orbit_bg", "heavy_tiles", "opaque_stack", "wide_strip_520_tiles"])
def test_backward_parity_exact(name):
    """The backward over an exact-mode forward replays its arithmetic (the mode recorded with the
    image buffer): every gradient within the same 1e-4 of the oracle.  faint_opacity puts
    alpha ~ 1/255 everywhere, opaque_stack saturates most pixels early."""
    _, _, _lib = _dgr()
    case = next(c for c in CASES if c["name"] == name)
    with _lib.exact_blend_mode():
        test_backward_parity(case)


def test_autograd_module_path():
    """The drop-in GaussianRasterizer as gaussian_renderer.render() uses it (colors_precomp,
    sh_degree=-1, scales/rotations, means2D with retain_grad)."""
    dgr, _, _ = _dgr()
    cam, gs = make_case(P=3000, W=96, H=96, sh_degree=0)
    dev = "cuda"
    s = dgr.GaussianRasterizationSettings(image_height=96, image_width=96, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
                                          bg=torch.zeros(3, device=dev), scale_modifier=1.0,
                                          viewmatrix=cam.world_view_transform.to(dev),
                                          projmatrix=cam.full_proj_transform.to(dev), sh_degree=-1,
                                          campos=cam.camera_center.to(dev), prefiltered=False)
    rast = dgr.GaussianRasterizer(raster_settings=s)
    leaves = {k: gs[k].to(dev).requires_grad_(True) for k in ("means3D", "colors", "opacities", "scales", "rotations")}
    means2D = torch.zeros_like(leaves["means3D"], requires_grad=True) + 0
    means2D.retain_grad()
    img, radii = rast(means3D=leaves["means3D"], means2D=means2D, shs=None, colors_precomp=leaves["colors"],
                      opacities=leaves["opacities"], scales=leaves["scales"], rotations=leaves["rotations"],
                      cov3D_precomp=None)
    assert img.shape == (3, 96, 96) and radii.shape == (3000,)
    (img * torch.linspace(0, 1, 96, device=dev)).sum().backward()
    for k, v in leaves.items():
        assert v.grad is not None and torch.isfinite(v.grad).all(), k
    assert means2D.grad is not None and (means2D.grad[:, :2].abs().sum() > 0)
    vis = rast.markVisible(leaves["means3D"].detach())
    assert vis.dtype == torch.bool and vis.all()  # every synthetic point is in front of the camera
    with pytest.raises(Exception):
        rast(means3D=leaves["means3D"], means2D=means2D, opacities=leaves["opacities"])


def test_empty_and_fully_culled():
    _, _C, _ = _dgr()
    cam, gs = make_case(P=100, W=32, H=32)
    dev = "cuda"
    e = torch.empty(0, device=dev)
    args = lambda m, c, o, s, r: (torch.zeros(3, device=dev), m, c, o, s, r, 1.0, e, cam.world_view_transform.cuda(),
                                  cam.full_proj_transform.cuda(), cam.tanfovx, cam.tanfovy, 32, 32, e, 0,
                                  cam.camera_center.cuda(), False)
    z = torch.zeros((0, 3), device=dev)
    R, color, radii, *_ = _C.rasterize_gaussians(*args(z, z, torch.zeros((0, 1), device=dev), z,
                                                       torch.zeros((0, 4), device=dev)))
    assert R == 0 and color.abs().max() == 0 and radii.numel() == 0
    behind = gs["means3D"].clone()
    behind[:, 2] = -behind[:, 2]
    R, color, radii, *_ = _C.rasterize_gaussians(*args(behind.cuda(), gs["colors"].cuda(), gs["opacities"].cuda(),
                                                       gs["scales"].cuda(), gs["rotations"].cuda()))
    assert R == 0 and (radii == 0).all() and color.abs().max() == 0


def test_prefiltered_error_is_reported():
    _, _C, _ = _dgr()
    cam, gs = make_case(P=64, W=32, H=32)
    behind = gs["means3D"].clone()
    behind[:5, 2] = -1.0
    dev = "cuda"
    e = torch.empty(0, device=dev)
    with pytest.raises(RuntimeError, match="prefiltered"):
        _C.rasterize_gaussians(torch.zeros(3, device=dev), behind.cuda(), gs["colors"].cuda(), gs["opacities"].cuda(),
                               gs["scales"].cuda(), gs["rotations"].cuda(), 1.0, e, cam.world_view_transform.cuda(),
                               cam.full_proj_transform.cuda(), cam.tanfovx, cam.tanfovy, 32, 32, e, 0,
                               cam.camera_center.cuda(), True)


def test_bad_means_shape():
    _, _C, _ = _dgr()
    dev = "cuda"
    e = torch.empty(0, device=dev)
    with pytest.raises(RuntimeError, match="means3D must have dimensions"):
        _C.rasterize_gaussians(torch.zeros(3, device=dev), torch.zeros(10, 4, device=dev), e, e, e, e, 1.0, e,
                               torch.eye(4, device=dev), torch.eye(4, device=dev), 1.0, 1.0, 8, 8, e, 0,
                               torch.zeros(3, device=dev), False)


@pytest.mark.parametrize("mode", ["colors_scales", "sh3_scales", "colors_cov3D"])
def test_autograd_node_matches_oracle_node(mode):
    """_RasterizeGaussians end to end against the same autograd node over the C oracle
    (oracle/oracle_torch.py, the reference's __init__.py:17-195 surface): every leaf
    gradient lands on the right input (means3D and means2D are both [P,3], so a swapped
    order would not show in shapes), with the reference's call pattern (means2D zeros + 0
    with retain_grad)."""
    from oracle import oracle_torch
    dgr, _, _ = _dgr()
    sh_deg = 3 if mode.startswith("sh3") else 0
    cam, gs = make_case(P=2500, W=80, H=64, sh_degree=sh_deg, camera="orbit")
    P = gs["means3D"].shape[0]
    g = torch.Generator().manual_seed(12)
    dout = torch.randn(3, 64, 80, generator=g)
    cov = None
    if mode == "colors_cov3D":
        cov = torch.from_numpy(orc.preprocess(np32(gs["means3D"]), np32(gs["scales"]), np32(gs["rotations"]),
                                              np32(gs["opacities"]).reshape(-1), None, np.zeros((P, 3), np.float32),
                                              None, np.eye(4, dtype=np.float32), np.eye(4, dtype=np.float32),
                                              np.zeros(3, np.float32), 16, 16, 1.0, 1.0, 1.0)["cov3D"])

    def run(mod, dev):
        s = mod.GaussianRasterizationSettings(
            image_height=64, image_width=80, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
            bg=torch.tensor([0.1, 0.2, 0.3], device=dev), scale_modifier=1.0,
            viewmatrix=cam.world_view_transform.to(dev), projmatrix=cam.full_proj_transform.to(dev),
            sh_degree=sh_deg if mode.startswith("sh3") else -1, campos=cam.camera_center.to(dev), prefiltered=False)
        lv = {"means3D": gs["means3D"], "opacities": gs["opacities"]}
        if mode.startswith("sh3"):
            lv["shs"] = gs["shs"]
        else:
            lv["colors_precomp"] = gs["colors"]
        if cov is None:
            lv.update(scales=gs["scales"], rotations=gs["rotations"])
        else:
            lv["cov3D_precomp"] = cov
        lv = {k: v.clone().to(dev).requires_grad_(True) for k, v in lv.items()}
        means2D = torch.zeros_like(lv["means3D"], requires_grad=True) + 0
        means2D.retain_grad()
        img, radii = mod.GaussianRasterizer(s)(means2D=means2D, **lv)
        (img * dout.to(dev)).sum().backward()
        grads = {k: v.grad.detach().cpu().numpy() for k, v in lv.items()}
        grads["means2D"] = means2D.grad.detach().cpu().numpy()
        return img.detach().cpu().numpy(), radii.cpu().numpy(), grads

    img, radii, grads = run(dgr, "cuda")
    w_img, w_radii, w_grads = run(oracle_torch, "cpu")
    assert np.array_equal(radii, w_radii)
    assert rel_l2(img, w_img) <= RGB_TOL
    assert sorted(grads) == sorted(w_grads)
    errs = {k: rel_l2(grads[k], w_grads[k]) for k in grads}
    assert all(e <= GRAD_TOL for e in errs.values()), errs


@pytest.mark.parametrize("camera", ["identity", "orbit"])
def test_mark_visible_matches_oracle(camera):
    """markVisible (rasterizer_impl.cu:54-66, rasterize_points.cu:194-213): present =
    (view * p).z > 0.2, bit-exact against orc_mark_visible on a cloud straddling the near
    plane and points behind the camera."""
    dgr, _C, _ = _dgr()
    cam, gs = make_case(P=6000, W=64, H=64, camera=camera)
    g = torch.Generator().manual_seed(5)
    pts = gs["means3D"].clone()
    pts[:2000, 2] = torch.rand(2000, generator=g) * 0.6 - 0.1  # around z = 0.2 (identity camera)
    pts[2000:2500] *= -1.0
    want = orc.mark_visible(np32(pts), np32(cam.world_view_transform))
    s = dgr.GaussianRasterizationSettings(image_height=64, image_width=64, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
                                          bg=torch.zeros(3, device="cuda"), scale_modifier=1.0,
                                          viewmatrix=cam.world_view_transform.cuda(),
                                          projmatrix=cam.full_proj_transform.cuda(), sh_degree=0,
                                          campos=cam.camera_center.cuda(), prefiltered=False)
    got = dgr.GaussianRasterizer(s).markVisible(pts.cuda()).cpu().numpy()
    assert got.dtype == bool and want.any() and not want.all()
    np.testing.assert_array_equal(got, want)
    got2 = _C.mark_visible(pts.cuda(), cam.world_view_transform.cuda(), cam.full_proj_transform.cuda()).cpu().numpy()
    np.testing.assert_array_equal(got2, want)


def test_speculative_binning_capacity_and_overflow():
    """The forward sizes its binning buffer from the previous call with the same P and image
    size and launches the binning before the host synchronisation (gsr_capi.cpp).  A call
    whose instance count exceeds that capacity (Gaussians 20x larger) must detect the
    overflow and redo the binning; the next, small, call runs in the oversized buffer.  Every
    call is checked against the oracle."""
    cam, gs = make_case(P=3000, W=96, H=80, sh_degree=0, camera="orbit")
    big = dict(gs, scales=gs["scales"] * 20.0)
    Rs = []
    for g in (gs, gs, big, gs, big):
        st = run_gpu(cam, g, mode="colors")
        ref = run_oracle(cam, g, mode="colors")
        check_forward(st, ref, 96, 80)
        Rs.append(st["R"])
    assert Rs[2] > 2 * Rs[1] and Rs[0] == Rs[1] == Rs[3]


def test_second_backward_over_one_forward():
    """The forward zeroes the gradient accumulators (inside the depth sort's digit scans) and
    the first backward skips its zero-fill; a second backward over the same buffers (autograd's
    retain_graph) must zero-fill again and return the same gradients."""
    _, _C, _ = _dgr()
    cam, gs = make_case(P=3000, W=128, H=96, sh_degree=2, camera="orbit")
    st = run_gpu(cam, gs, mode="sh", sh_degree=2)
    W, H = cam.image_width, cam.image_height
    dout = torch.randn(3, H, W, generator=torch.Generator().manual_seed(4)).cuda()

    def bwd():
        return _C.rasterize_gaussians_backward(
            st["bg"], st["means"], st["radii"], st["colors"], st["scales"], st["rots"], 1.0, st["cov3"], st["vm"],
            st["pm"], cam.tanfovx, cam.tanfovy, dout, st["sh"], 2, st["cp"], st["geom"], st["R"], st["binb"],
            st["img"])
    g1 = [t.clone() for t in bwd()]
    g2 = bwd()
    for a, b in zip(g1, g2):
        if a.numel():
            assert rel_l2(b.cpu().numpy(), a.cpu().numpy()) < 1e-6


@pytest.mark.parametrize("mode", ["sh", "colors"])
def test_backward_skips_unneeded_outputs(mode):
    """colors_grad / cov3D_grad = False (what the autograd node passes for an empty
    colors_precomp / cov3D_precomp): dL_dcolors and dL_dcov3D come back as None, the other six
    outputs bit-equal to the reference's full output set (deterministic mode: fixed-order sums);
    through GaussianRasterizer the SH path's gradients are unchanged."""
    dgr, _C, _lib = _dgr()
    cam, gs = make_case(P=3000, W=96, H=80, sh_degree=2 if mode == "sh" else 0, camera="orbit")
    kw = dict(mode=mode, sh_degree=2 if mode == "sh" else 0)
    W, H = cam.image_width, cam.image_height
    dout = torch.randn(3, H, W, generator=torch.Generator().manual_seed(4)).cuda()
    _lib.set_deterministic(True)
    try:
        st = run_gpu(cam, gs, **kw)
        args = (st["bg"], st["means"], st["radii"], st["colors"], st["scales"], st["rots"], 1.0, st["cov3"], st["vm"],
                st["pm"], cam.tanfovx, cam.tanfovy, dout, st["sh"], kw["sh_degree"], st["cp"], st["geom"], st["R"],
                st["binb"], st["img"])
        full = _C.rasterize_gaussians_backward(*args)
        part = _C.rasterize_gaussians_backward(*args, colors_grad=False, cov3D_grad=False)
    finally:
        _lib.set_deterministic(False)
    assert part[1] is None and part[4] is None
    assert full[1] is not None and full[4] is not None and full[4].abs().max() > 0
    for i in (0, 2, 3, 5, 6, 7):
        assert torch.equal(part[i], full[i]), i
    if mode == "sh":  # the autograd node passes the flags: gradients unchanged against the full call
        dev = torch.device("cuda")
        leaves = {k: gs[k].to(dev).requires_grad_(True) for k in ("means3D", "shs", "opacities", "scales", "rotations")}
        means2D = torch.zeros_like(leaves["means3D"], requires_grad=True)
        s = dgr.GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, bg=st["bg"], scale_modifier=1.0,
            viewmatrix=st["vm"], projmatrix=st["pm"], sh_degree=kw["sh_degree"], campos=st["cp"], prefiltered=False)
        img, _ = dgr.GaussianRasterizer(s)(means3D=leaves["means3D"], means2D=means2D, shs=leaves["shs"],
                                           opacities=leaves["opacities"], scales=leaves["scales"],
                                           rotations=leaves["rotations"])
        (img * dout).sum().backward()
        for got, ref in ((means2D.grad, full[0]), (leaves["means3D"].grad, full[3]), (leaves["shs"].grad, full[5]),
                         (leaves["scales"].grad, full[6]), (leaves["rotations"].grad, full[7])):
            assert rel_l2(got.cpu().numpy(), ref.cpu().numpy()) < 1e-5
