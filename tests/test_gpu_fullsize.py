"""GPU parity at BASELINE.json's full size (cfg2: 1.5M Gaussians, SH3, 1920x1080).

The oracle cannot bin and render 28M instances in seconds, so the full-size checks are:
  * every per-Gaussian preprocess output bit-exact against the C oracle (all 1.5M);
  * size-independent binning invariants: tile ranges partition [0, R) in tile order, every
    Gaussian appears in exactly tiles_touched lists, each list is sorted by (depth, index)
    and only names Gaussians whose rect covers the tile;
  * sampled parity: the oracle renders 32 random tiles from the GPU's own lists and records,
    forward colours/T/n_contrib compared there; the backward is run with dL/dpix zero outside
    those tiles, so the full GPU gradients must equal the oracle's for the same tiles;
  * backward linearity in dL/dpix and bit-identical repeated forwards.
"""
import numpy as np
import pytest
import torch

from helpers import np32, rel_l2
from oracle import oracle as orc
from test_gpu_rasterizer import run_gpu

pytestmark = pytest.mark.gpu

TILE_SAMPLE = 32


@pytest.fixture(scope="module")
def cfg2():
    from gsr import scenes
    cam, gs, c = scenes.build_config("cfg2", device="cpu", seed=0)
    st = run_gpu(cam, gs, mode="sh", sh_degree=c["sh_degree"])
    return cam, gs, c, st


def _grads(cam, gs, st, dout, deg):
    from diff_gaussian_rasterization import _C
    return _C.rasterize_gaussians_backward(st["bg"], st["means"], st["radii"], st["colors"], st["scales"], st["rots"],
                                           1.0, st["cov3"], st["vm"], st["pm"], cam.tanfovx, cam.tanfovy, dout,
                                           st["sh"], deg, st["cp"], st["geom"], st["R"], st["binb"], st["img"])


def test_cfg2_preprocess_bit_exact(cfg2):
    cam, gs, c, st = cfg2
    W, H = cam.image_width, cam.image_height
    ref = orc.preprocess(np32(gs["means3D"]), np32(gs["scales"]), np32(gs["rotations"]),
                         np32(gs["opacities"]).reshape(-1), np32(gs["shs"]), None, None, np32(cam.world_view_transform),
                         np32(cam.full_proj_transform), np32(cam.camera_center), W, H, cam.tanfovx, cam.tanfovy, 1.0,
                         c["sh_degree"])
    vis = ref["radii"] > 0
    assert vis.sum() > 1_000_000
    np.testing.assert_array_equal(st["radii"].cpu().numpy(), ref["radii"])
    np.testing.assert_array_equal(st["tiles"], ref["tiles_touched"])
    rec = st["rec"]
    np.testing.assert_array_equal(rec[vis, 0:2], ref["means2D"][vis])
    np.testing.assert_array_equal(rec[vis, 2:6], ref["conic_opacity"][vis])
    np.testing.assert_array_equal(rec[vis, 6:9], ref["rgb"][vis])
    np.testing.assert_array_equal(st["depth_key"][vis], ref["depths"][vis].view(np.uint32))


def test_cfg2_binning_invariants(cfg2):
    cam, gs, c, st = cfg2
    W, H = cam.image_width, cam.image_height
    gx, gy = (W + 15) // 16, (H + 15) // 16
    R, pl, rg = st["R"], st["point_list"].astype(np.int64), st["ranges"].astype(np.int64)
    P = gs["means3D"].shape[0]
    assert R == int(st["tiles"].astype(np.int64).sum()) and R > 10_000_000
    lens = rg[:, 1] - rg[:, 0]
    assert (lens >= 0).all() and lens.sum() == R
    ne = lens > 0
    # non-empty ranges are consecutive in tile order and cover [0, R)
    starts, ends = rg[ne, 0], rg[ne, 1]
    assert starts[0] == 0 and ends[-1] == R and (starts[1:] == ends[:-1]).all()
    # each Gaussian is listed exactly tiles_touched times
    np.testing.assert_array_equal(np.bincount(pl, minlength=P), st["tiles"].astype(np.int64))
    # lists sorted by (depth bits, index) within every tile
    tile_of = np.repeat(np.arange(gx * gy), lens)
    key = st["depth_key"].astype(np.uint64)[pl]
    same = tile_of[1:] == tile_of[:-1]
    k0, k1 = key[:-1][same], key[1:][same]
    i0, i1 = pl[:-1][same], pl[1:][same]
    assert ((k0 < k1) | ((k0 == k1) & (i0 < i1))).all()
    # every listed Gaussian's rect (forward.cu getRect) covers its tile
    rec = st["rec"]
    rad = st["radii"].cpu().numpy().astype(np.int64)
    x, y = rec[pl, 0], rec[pl, 1]
    r = rad[pl].astype(np.float32)
    tx, ty = tile_of % gx, tile_of // gx
    f16, f1 = np.float32(16), np.float32(1)
    # float32 arithmetic in the reference's order, truncating casts (forward.cu getRect)
    xmin = np.clip(((x - r) / f16).astype(np.int64), 0, gx)
    xmax = np.clip(((((x + r) + f16) - f1) / f16).astype(np.int64), 0, gx)
    ymin = np.clip(((y - r) / f16).astype(np.int64), 0, gy)
    ymax = np.clip(((((y + r) + f16) - f1) / f16).astype(np.int64), 0, gy)
    inside = (tx >= xmin) & (tx < xmax) & (ty >= ymin) & (ty < ymax)
    assert inside.all(), inside.mean()


def _sample_tiles(gx, gy, seed=5):
    return np.random.default_rng(seed).choice(gx * gy, size=TILE_SAMPLE, replace=False).astype(np.int32)


def _tile_mask(tiles, gx, W, H):
    m = np.zeros((H, W), bool)
    for t in tiles:
        bx, by = int(t) % gx, int(t) // gx
        m[by * 16:min(by * 16 + 16, H), bx * 16:min(bx * 16 + 16, W)] = True
    return m


def test_cfg2_sampled_tiles_forward(cfg2):
    cam, gs, c, st = cfg2
    W, H = cam.image_width, cam.image_height
    gx, gy = (W + 15) // 16, (H + 15) // 16
    tiles = _sample_tiles(gx, gy)
    rec = st["rec"]
    out, fT, nc = orc.render_fwd(st["ranges"], st["point_list"], rec[:, 0:2], rec[:, 6:9], rec[:, 2:6],
                                 np.zeros(3, np.float32), W, H, tiles=tiles)
    m = _tile_mask(tiles, gx, W, H)
    color = st["color"].cpu().numpy()
    assert rel_l2(color[:, m], out[:, m]) <= 1e-4
    assert (st["n_contrib"].reshape(H, W)[m] == nc.reshape(H, W)[m]).mean() > 0.999
    assert rel_l2(st["final_T"].reshape(H, W)[m], fT.reshape(H, W)[m]) <= 1e-4


def test_cfg2_sampled_tiles_backward(cfg2):
    cam, gs, c, st = cfg2
    W, H = cam.image_width, cam.image_height
    gx, gy = (W + 15) // 16, (H + 15) // 16
    P = gs["means3D"].shape[0]
    tiles = _sample_tiles(gx, gy)
    m = _tile_mask(tiles, gx, W, H)
    dout = np.random.default_rng(9).standard_normal((3, H, W)).astype(np.float32) * m[None]
    g = _grads(cam, gs, st, torch.tensor(dout, device="cuda"), c["sh_degree"])
    torch.cuda.synchronize()
    rec = st["rec"]
    bg = np.zeros(3, np.float32)
    _, fT, nc = orc.render_fwd(st["ranges"], st["point_list"], rec[:, 0:2], rec[:, 6:9], rec[:, 2:6], bg, W, H,
                               tiles=tiles)
    rb = orc.render_bwd(P, st["ranges"], st["point_list"], bg, rec[:, 0:2], rec[:, 2:6], rec[:, 6:9], fT, nc, dout, W,
                        H, tiles=tiles)
    fwd = orc.preprocess(np32(gs["means3D"]), np32(gs["scales"]), np32(gs["rotations"]),
                         np32(gs["opacities"]).reshape(-1), np32(gs["shs"]), None, None, np32(cam.world_view_transform),
                         np32(cam.full_proj_transform), np32(cam.camera_center), W, H, cam.tanfovx, cam.tanfovy, 1.0,
                         c["sh_degree"])
    fwd["cov3D_used"] = fwd["cov3D"]
    pb = orc.preprocess_bwd(fwd, np32(gs["means3D"]), np32(gs["shs"]), c["sh_degree"], np32(gs["scales"]),
                            np32(gs["rotations"]), 1.0, np32(cam.world_view_transform),
                            np32(cam.full_proj_transform), W, H, cam.tanfovx, cam.tanfovy, np32(cam.camera_center),
                            rb["dL_dmean2D"], rb["dL_dconic"], rb["dL_dcolors"])
    ref = [rb["dL_dmean2D"], rb["dL_dcolors"], rb["dL_dopacity"], pb["dL_dmeans3D"], pb["dL_dcov3D"], pb["dL_dsh"],
           pb["dL_dscales"], pb["dL_drotations"]]
    names = ["dmean2D", "dcolors", "dopacity", "dmeans3D", "dcov3D", "dsh", "dscales", "drot"]
    touched = np.abs(rb["dL_dopacity"]).reshape(-1) > 0
    assert touched.sum() > 1000
    for n, mine, r in zip(names, g, ref):
        mine = mine.detach().cpu().numpy().reshape(r.shape)
        if np.abs(r).max() == 0:
            continue
        assert rel_l2(mine, r) <= 1e-4, (n, rel_l2(mine, r))


def test_cfg2_backward_linear_in_dpix(cfg2):
    cam, gs, c, st = cfg2
    W, H = cam.image_width, cam.image_height
    gen = torch.Generator(device="cuda").manual_seed(3)
    d1 = torch.randn(3, H, W, device="cuda", generator=gen)
    d2 = torch.randn(3, H, W, device="cuda", generator=gen)
    g1 = _grads(cam, gs, st, d1, c["sh_degree"])
    g2 = _grads(cam, gs, st, d2, c["sh_degree"])
    g12 = _grads(cam, gs, st, d1 + d2, c["sh_degree"])
    for a, b, s in zip(g1, g2, g12):
        if s.numel() == 0:
            continue
        s_ = s.double()
        assert (torch.linalg.norm((a.double() + b.double()) - s_) / torch.linalg.norm(s_).clamp_min(1e-30)) < 1e-4


def test_forward_is_deterministic(cfg2):
    cam, gs, c, st = cfg2
    st2 = run_gpu(cam, gs, mode="sh", sh_degree=c["sh_degree"])
    assert torch.equal(st["color"], st2["color"])
    np.testing.assert_array_equal(st["point_list"], st2["point_list"])
    np.testing.assert_array_equal(st["n_contrib"], st2["n_contrib"])


@pytest.mark.parametrize("W,H,P", [(3840, 2160, 100_000), (5120, 2880, 60_000)])
def test_large_frame_binning_exact(W, H, P):
    """cfg5's 3840x2160 frame: 30 x 34 = 1020 super-tiles run the fused
    super-tile binning with four waves per workgroup (eight would exceed its LDS budget);
    5120x2880 (1800 super-tiles) exceeds that too and runs the emit + offsets scan +
    one-pass sort path.  Both must reproduce the oracle's (tile, depth, index) lists and
    tile ranges bit for bit."""
    from gsr import scenes
    cam, gs, c = scenes.build_config("cfg5", device="cpu", seed=1, P=P, W=W, H=H)
    st = run_gpu(cam, gs, mode="sh", sh_degree=c["sh_degree"])
    ref = orc.preprocess(np32(gs["means3D"]), np32(gs["scales"]), np32(gs["rotations"]),
                         np32(gs["opacities"]).reshape(-1), np32(gs["shs"]), None, None, np32(cam.world_view_transform),
                         np32(cam.full_proj_transform), np32(cam.camera_center), W, H, cam.tanfovx, cam.tanfovy, 1.0,
                         c["sh_degree"])
    R, keys, vals, ranges = orc.binning(ref, W, H)
    assert st["R"] == R and R > 500_000
    np.testing.assert_array_equal(st["point_list"].astype(np.int64), vals.astype(np.int64))
    np.testing.assert_array_equal(st["ranges"].astype(np.int64), ranges.astype(np.int64))
