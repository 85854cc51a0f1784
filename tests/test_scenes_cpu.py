"""The Trevi-class clustered workload (gsr.scenes.trevi_like_gaussians, cfg2c) on the CPU:
its construction (quaternions, sky band, determinism) and the load features it exists for
(culling, heavy tiles), checked with the C oracle's preprocess and binning."""
import math

import numpy as np
import torch

from gsr import scenes
from oracle import oracle as orc


def test_rotmat_to_quat_round_trip():
    rng = np.random.default_rng(0)
    q = rng.normal(size=(500, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    r, x, y, z = q.T
    # build_rotation (utils/general_utils.py:98-119)
    Rm = np.stack([np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], 1),
                   np.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], 1),
                   np.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], 1)], 1)
    q2 = scenes._rotmat_to_quat(Rm)
    # q and -q are the same rotation
    assert np.allclose(np.abs((q * q2).sum(1)), 1.0, atol=1e-9)


def test_trevi_structure_and_determinism():
    P = 60_000
    a = scenes.trevi_like_gaussians(P, sh_degree=3, seed=0)
    b = scenes.trevi_like_gaussians(P, sh_degree=3, seed=0)
    for k in a:
        assert torch.equal(a[k], b[k]), k
    assert a["means3D"].shape == (P, 3) and a["shs"].shape == (P, 16, 3)
    assert int(a["is_sky"].sum()) == P // 10
    assert torch.allclose(a["rotations"].norm(dim=1), torch.ones(P), atol=1e-5)
    op = a["opacities"].reshape(-1)
    assert float(op.min()) > 0 and float(op.max()) < 1
    assert float((op[~a["is_sky"]] > 0.9).float().mean()) > 0.45  # skewed high, as trained
    # the sky band of sample_points_on_unit_hemisphere around the camera centre: elevation
    # 0..30 degrees (COLMAP -y up), azimuth within +-45 degrees, one radius
    s = a["means3D"][a["is_sky"]].double()
    rad = s.norm(dim=1)
    assert float(rad.max() - rad.min()) < 1e-3 * float(rad.mean())
    assert float(s[:, 1].max()) <= 1e-6 and float((-s[:, 1] / rad).max()) <= 0.5 + 1e-6
    assert float(torch.atan2(s[:, 0], s[:, 2]).abs().max()) <= math.pi / 4 + 1e-6


def test_trevi_culls_and_has_heavy_tiles():
    """At a tenth of cfg2c's size: a real culled fraction, and tiles whose lists are far longer
    than the median (the load imbalance the uniform cfg2 cloud lacks)."""
    cam, gs, c = scenes.build_config("cfg2c", P=150_000)
    W, H = cam.image_width, cam.image_height
    n = lambda k: gs[k].numpy()
    pre = orc.preprocess(n("means3D"), n("scales"), n("rotations"), n("opacities").reshape(-1), n("shs"), None, None,
                         cam.world_view_transform.numpy(), cam.full_proj_transform.numpy(),
                         cam.camera_center.numpy(), W, H, cam.tanfovx, cam.tanfovy, 1.0, 3)
    vis = pre["radii"] > 0
    culled = 1 - vis.mean()
    assert 0.1 < culled < 0.35, culled
    assert 0.5 < vis[n("is_sky")].mean() < 0.95  # part of the sky band is outside the frame
    R, _, _, ranges = orc.binning(pre, W, H)
    lens = ranges[:, 1].astype(np.int64) - ranges[:, 0]
    assert lens.max() > 3 * max(np.median(lens), 1), (lens.max(), np.median(lens))
