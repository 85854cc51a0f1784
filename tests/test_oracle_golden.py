"""Pin the CPU oracle (oracle/gsr_oracle.c) against golden vectors produced by importing the
reference's own Python (tools/gen_golden.py).  CPU only."""
import os

import numpy as np
import pytest

from oracle import oracle as orc


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


@pytest.mark.parametrize("deg", range(6))
def test_eval_sh_matches_reference(golden_dir, deg):
    g = load(golden_dir, "eval_sh.npz")
    sh = g[f"sh{deg}"]  # [N, 3, K] reference layout
    out = orc.eval_sh(deg, np.transpose(sh, (0, 2, 1)), g[f"dirs{deg}"])
    np.testing.assert_allclose(out, g[f"out{deg}"], rtol=2e-5, atol=2e-6)


def test_cov3d_matches_reference_python(golden_dir):
    """forward.cu:118-152 computeCov3D vs gaussian_model.py:30-34 (normalised quaternions)."""
    g = load(golden_dir, "geometry.npz")
    P = g["scales"].shape[0]
    view = np.eye(4, dtype=np.float32)
    geom = orc.preprocess(g["xyz"], g["scales"], g["rotations"], np.full(P, 0.5, np.float32), None,
                          np.zeros((P, 3), np.float32), None, view, view, np.zeros(3, np.float32), 64, 64, 1.0,
                          1.0, scale_modifier=float(g["scale_modifier"]))
    vis = geom["radii"] > 0
    assert vis.sum() > P // 2
    ref = g["cov3D"]
    scale = np.abs(ref).max(axis=1, keepdims=True)
    assert np.all(np.abs(geom["cov3D"][vis] - ref[vis]) <= 2e-6 * scale[vis] + 1e-12)


@pytest.mark.parametrize("ci", range(3))
def test_depth_and_cameras_match_reference(golden_dir, ci):
    from gsr import scenes
    g = load(golden_dir, "geometry.npz")
    fovx, fovy = g[f"cam{ci}/fov"]
    W, H = (int(x) for x in g[f"cam{ci}/wh"])
    cam = scenes.make_camera(W, H, fovx, fovy, R=g[f"cam{ci}/R"], T=g[f"cam{ci}/T"])
    np.testing.assert_array_equal(cam.world_view_transform.numpy(), g[f"cam{ci}/viewmatrix"])
    np.testing.assert_array_equal(cam.full_proj_transform.numpy(), g[f"cam{ci}/projmatrix"])
    np.testing.assert_array_equal(cam.camera_center.numpy(), g[f"cam{ci}/campos"])
    xyz = g["xyz"]
    P = xyz.shape[0]
    geom = orc.preprocess(xyz, g["scales"], g["rotations"], np.full(P, 0.5, np.float32), None,
                          np.zeros((P, 3), np.float32), None, g[f"cam{ci}/viewmatrix"], g[f"cam{ci}/projmatrix"],
                          g[f"cam{ci}/campos"], W, H, np.tan(fovx / 2), np.tan(fovy / 2))
    vis = geom["radii"] > 0
    assert vis.any()
    np.testing.assert_allclose(geom["depths"][vis], g[f"cam{ci}/depth"][vis, 0], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("deg", range(4))
def test_sh_to_rgb_matches_reference(golden_dir, deg):
    """forward.cu:20-71 computeColorFromSH vs eval_sh + 0.5 clamp."""
    g = load(golden_dir, "geometry.npz")
    xyz = g["xyz"]
    P = xyz.shape[0]
    view = np.eye(4, dtype=np.float32)
    K = (deg + 1) ** 2
    shs = np.ascontiguousarray(g[f"shrgb{deg}/shs"][:, :K, :])
    geom = orc.preprocess(xyz, g["scales"], g["rotations"], np.full(P, 0.5, np.float32), shs, None, None, view,
                          view, g[f"shrgb{deg}/campos"], 64, 64, 1.0, 1.0, sh_degree=deg)
    vis = geom["radii"] > 0
    np.testing.assert_allclose(geom["rgb"][vis], g[f"shrgb{deg}/rgb"][vis], rtol=1e-5, atol=2e-6)


SHADE_CASES = ["spec_km", "spec_nokm", "diffuse", "spec_km_deg5", "spec_km_deg2"]


def _lut():
    from gsr import assets
    return assets.load_fg_lut()


@pytest.mark.parametrize("case", SHADE_CASES)
def test_shade_forward_matches_reference(golden_dir, case):
    g = load(golden_dir, "shade.npz")
    f = lambda k: g[f"{case}/{k}"]
    km = f("km") if bool(f("with_km")) else None
    rgb, dif, spe = orc.shade_fwd(f("pos"), f("normal"), f("albedo"), f("view_pos"), f("kr"), km, f("base"), _lut(),
                                  deg=int(f("deg")), specular=bool(f("specular")))
    np.testing.assert_allclose(rgb, f("rgb"), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(dif, f("diffuse"), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(spe, f("specular_out"), rtol=1e-5, atol=1e-6)


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


@pytest.mark.parametrize("case", SHADE_CASES)
def test_shade_backward_matches_reference_autograd(golden_dir, case):
    g = load(golden_dir, "shade.npz")
    f = lambda k: g[f"{case}/{k}"]
    with_km = bool(f("with_km"))
    km = f("km") if with_km else None
    d = orc.shade_bwd(f("pos"), f("normal"), f("albedo"), f("view_pos"), f("kr"), km, f("base"), _lut(),
                      f("g_rgb"), f("g_diffuse"), f("g_specular"), deg=int(f("deg")), specular=bool(f("specular")))
    pairs = [("pos", "d_pos"), ("normal", "d_normal"), ("albedo", "d_albedo"), ("view_pos", "d_view_pos"),
             ("kr", "d_kr"), ("base", "d_base")]
    if with_km:
        pairs.append(("km", "d_km"))
    for mine, ref in pairs:
        r = f(ref)
        if r.size == 0:
            assert np.abs(d[mine]).max() == 0.0, mine
            continue
        e = rel_err(d[mine].reshape(r.shape), r)
        assert e < 1e-5, (mine, e)
