"""CPU: the sky Gaussians' parametrisation and densification in gsr.train / gsr.densify
against fixtures the reference's own Python produced (tests/golden/train_sky.npz,
tools/gen_golden_train.py):

  * get_xyz with (theta, phi) sky rows interleaved among the foreground rows, angles outside
    the admitted range clamped, and its gradients to the foreground xyz, the angles and the
    shell radius (scene/gaussian_model.py:84-103,159-169);
  * cartesian_to_polar_coord with the default and an explicit radius
    (utils/general_utils.py:295-299);
  * densify_and_prune on a scene with an Adam state: clone, split (sky samples projected
    onto the shell and turned back into angles with the default radius of 1, :571-573),
    prune -- every group's rows and both Adam moments (gaussian_model.py:438-625).

Tolerances: 1e-6 relative (the same fp32 operations; the split's samples are drawn from a
generator seeded as the reference's global RNG was)."""
import os

import numpy as np
import pytest
import torch

from helpers import rel_l2

GOLD = os.path.join(os.path.dirname(__file__), "golden", "train_sky.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def test_get_xyz_and_gradients(gold):
    from gsr import train
    is_sky = torch.tensor(gold["sky/is_sky"])
    lay = train.SkyLayout(is_sky)
    assert not lay.tail and lay.n_sky == int(is_sky.sum())
    xyz = torch.tensor(gold["sky/xyz_fg"]).requires_grad_(True)
    ang = torch.tensor(gold["sky/angles"]).requires_grad_(True)
    rad = torch.tensor([float(gold["sky/radius"])]).requires_grad_(True)
    center = torch.tensor(gold["sky/center"])
    out = lay.xyz(xyz, train.sky_xyz(ang, rad, center))
    assert rel_l2(out.detach().numpy(), gold["sky/get_xyz"]) < 1e-6
    dx, da, dr = torch.autograd.grad(out, [xyz, ang, rad], torch.tensor(gold["sky/g"]))
    assert rel_l2(dx.numpy(), gold["sky/d_xyz_fg"]) < 1e-6
    assert rel_l2(da.numpy(), gold["sky/d_angles"]) < 1e-6
    assert abs(float(dr) - float(gold["sky/d_radius"])) <= 1e-5 * abs(float(gold["sky/d_radius"]))
    # clamped angles get no gradient
    a = gold["sky/angles"]
    outside = (a[:, 0] < 0) | (a[:, 0] > np.pi / 2)
    assert outside.any() and np.all(da.numpy()[outside, 0] == 0)


def test_tail_layout_is_a_concatenation():
    from gsr import train
    is_sky = torch.zeros(10, dtype=torch.bool)
    is_sky[7:] = True
    lay = train.SkyLayout(is_sky)
    assert lay.tail
    a, b = torch.randn(7, 3), torch.randn(3, 3)
    assert torch.equal(lay.xyz(a, b), torch.cat([a, b]))
    lay2 = train.SkyLayout(is_sky[torch.tensor([0, 7, 1, 2, 8, 3, 4, 9, 5, 6])])
    assert not lay2.tail


def test_cartesian_to_polar(gold):
    from gsr import train
    pts, c = torch.tensor(gold["c2p/pts"]), torch.tensor(gold["c2p/center"])
    assert rel_l2(train.cartesian_to_polar_coord(pts, c).numpy(), gold["c2p/default_radius"]) < 1e-6
    assert rel_l2(train.cartesian_to_polar_coord(pts, c, 7.5).numpy(), gold["c2p/radius_7_5"]) < 1e-6


def _scene_from(gold):
    """A CPU RelitScene holding the fixture's rows and Adam moments."""
    from gsr import train
    is_sky = torch.tensor(gold["dens/before/is_sky"]).reshape(-1)
    P, n_fg = is_sky.numel(), int((~is_sky).sum())
    xyz = torch.zeros(P, 3)
    xyz[~is_sky] = torch.tensor(gold["dens/before/xyz"])
    xyz[is_sky] = 1.0  # replaced by the fixture's angles below
    b = lambda n: torch.tensor(gold[f"dens/before/{n}"])
    scene = train.RelitScene(xyz, b("scaling"), b("rotation"), b("opacity"), b("albedo"), b("roughness"),
                             b("metalness"), is_sky, 2, "cpu", sky_center=torch.tensor(gold["dens/center"]),
                             sky_radius=float(gold["dens/before/sky_radius"]))
    fp = scene.fp
    for n in train.GAUSSIAN_GROUPS:
        name = n[0]
        fp.load(name, b(name))
        off = fp.offsets[fp.names.index(name)]
        k = fp.params[name].numel()
        fp.exp_avg[off:off + k] = torch.tensor(gold[f"dens/before/m/{name}"]).reshape(-1)
        fp.exp_avg_sq[off:off + k] = torch.tensor(gold[f"dens/before/v/{name}"]).reshape(-1)
    scene.stats = {"xyz_gradient_accum": torch.tensor(gold["dens/accum"]), "denom": torch.tensor(gold["dens/denom"]),
                   "max_radii2D": torch.tensor(gold["dens/max_radii2D"])}
    assert n_fg == fp.params["xyz"].shape[0]
    return scene


def test_densify_and_prune_matches_reference(gold):
    from gsr import densify, train
    scene = _scene_from(gold)
    max_grad, min_opacity, extent, max_screen = (float(x) for x in gold["dens/args"])
    gen = torch.Generator().manual_seed(int(gold["dens/seed"]))
    densify.densify_and_prune(scene, max_grad, min_opacity, extent, max_screen, generator=gen)
    want_sky = gold["dens/after/is_sky"].reshape(-1)
    assert np.array_equal(scene.is_sky.reshape(-1).numpy(), want_sky)
    fp = scene.fp
    for name, _, _ in train.GAUSSIAN_GROUPS:
        want = gold[f"dens/after/{name}"]
        got = fp.params[name].detach().numpy()
        assert got.size == want.size, (name, got.shape, want.shape)
        assert rel_l2(got.reshape(want.shape), want) < 1e-6, name
        off = fp.offsets[fp.names.index(name)]
        k = got.size
        assert rel_l2(fp.exp_avg[off:off + k].numpy(), gold[f"dens/after/m/{name}"].reshape(-1)) < 1e-6, name
        assert rel_l2(fp.exp_avg_sq[off:off + k].numpy(), gold[f"dens/after/v/{name}"].reshape(-1)) < 1e-6, name
    assert rel_l2(scene.get_xyz().detach().numpy(), gold["dens/after/get_xyz"]) < 1e-6
    # the fixture exercises every branch: sky clones and splits, foreground clones and splits
    assert want_sky.sum() != gold["dens/before/is_sky"].sum() and (~want_sky).sum() != (~gold["dens/before/is_sky"]).sum()
