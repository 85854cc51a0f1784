"""CPU checks of gsr.relit's PyTorch restatements against the reference's own outputs:
eval_sh (utils/sh_utils.py:81-125, degrees 0-3; tests/golden/eval_sh.npz) -- the sky
colour of render_calls."""
import os

import numpy as np
import pytest
import torch

from gsr import relit

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_eval_sh_matches_reference(deg):
    d = np.load(os.path.join(GOLD, "eval_sh.npz"), allow_pickle=False)
    out = relit.eval_sh(deg, torch.from_numpy(d[f"sh{deg}"]), torch.from_numpy(d[f"dirs{deg}"]))
    np.testing.assert_allclose(out.numpy(), d[f"out{deg}"], rtol=1e-6, atol=1e-6)


def test_depth_to_normal_plane():
    """graphics_utils.py:158-169 on a fronto-parallel plane at depth 2 (identity camera):
    the inner normals are (0, 0, -1), the one-pixel border stays 0."""
    import types
    from gsr import scenes
    cam = scenes.make_camera(32, 24, 1.0, 0.8)
    view = types.SimpleNamespace(world_view_transform=cam.world_view_transform, image_width=32, image_height=24,
                                 FoVx=cam.FoVx, FoVy=cam.FoVy)
    n = relit.depth_to_normal(view, torch.full((1, 24, 32), 2.0))
    assert n.shape == (24, 32, 3)
    np.testing.assert_allclose(n[1:-1, 1:-1].numpy(), np.broadcast_to([0.0, 0.0, -1.0], (22, 30, 3)), atol=1e-6)
    assert not n[0].any() and not n[:, 0].any()


def test_depths_to_points_matches_reference_formula():
    """The broadcast form of graphics_utils.py:141-156 equals the reference's matrix form
    (pixels @ K^-1^T @ R^T) to float rounding on a rotated, translated camera."""
    import math
    import types
    from gsr import scenes
    R, T = scenes.look_at_rotation([0.5, 0.2, -1.0], [0.0, 0.0, 5.0])
    cam = scenes.make_camera(64, 48, 1.0, 0.8, R=R, T=T)
    view = types.SimpleNamespace(world_view_transform=cam.world_view_transform, image_width=64, image_height=48,
                                 FoVx=cam.FoVx, FoVy=cam.FoVy)
    d = torch.rand(1, 48, 64, generator=torch.Generator().manual_seed(0)) + 1
    c2w = view.world_view_transform.T.inverse()
    fx, fy = 64 / (2 * math.tan(view.FoVx / 2.)), 48 / (2 * math.tan(view.FoVy / 2.))
    K = torch.tensor([[fx, 0., 32.], [0., fy, 24.], [0., 0., 1.0]]).float()
    gx, gy = torch.meshgrid(torch.arange(64).float(), torch.arange(48).float(), indexing="xy")
    pts = torch.stack([gx, gy, torch.ones_like(gx)], dim=-1).reshape(-1, 3)
    ref = d.reshape(-1, 1) * (pts @ K.inverse().T @ c2w[:3, :3].T) + c2w[:3, 3]
    np.testing.assert_allclose(relit.depths_to_points(view, d).numpy(), ref.numpy(), rtol=1e-6, atol=1e-6)


def test_fg_index_cache_across_views():
    """relit_features' foreground index is rebuilt only when the sky flags change: render()
    hands it a fresh squeeze() view of the model's flags every call (a cache miss there is a
    nonzero + host synchronisation per view)."""
    import relit_shade as rs
    flags = torch.zeros(10, 1, dtype=torch.bool)
    flags[7:] = True
    cpu = torch.device("cpu")
    rows, rank = rs._fg_index(flags.squeeze(), 10, cpu)
    assert rows.tolist() == list(range(7)) and rank.tolist() == list(range(7)) + [-1] * 3
    again = rs._fg_index(flags.squeeze(), 10, cpu)
    assert again[0] is rows and again[1] is rank
    flags[0] = True  # in-place change (densification): version bump -> rebuilt
    rows2, rank2 = rs._fg_index(flags.squeeze(), 10, cpu)
    assert rows2.tolist() == list(range(1, 7)) and rank2.tolist() == [-1, 0, 1, 2, 3, 4, 5, -1, -1, -1]


def test_depth_to_normal_matches_reference_fixture():
    """gsr.relit.depth_to_normal against the reference's own depth_to_normal
    (utils/graphics_utils.py:141-169) on the reference Camera of tests/golden/render.npz,
    forward and depth gradient (tools/gen_golden_render.py)."""
    import types
    d = np.load(os.path.join(GOLD, "render.npz"), allow_pickle=False)
    view = types.SimpleNamespace(world_view_transform=torch.from_numpy(d["world_view_transform"]),
                                 image_width=int(d["W"]), image_height=int(d["H"]), FoVx=float(d["FoVx"]),
                                 FoVy=float(d["FoVy"]))
    depth = torch.from_numpy(d["d2n/depth"]).requires_grad_(True)
    n = relit.depth_to_normal(view, depth)
    np.testing.assert_allclose(n.detach().numpy(), d["d2n/normal"], rtol=0, atol=2e-5)
    w = np.random.default_rng(1099).standard_normal(tuple(n.shape)).astype(np.float32)
    (n * torch.from_numpy(w)).sum().backward()
    g, want = depth.grad.numpy(), d["d2n/grad_depth"]
    assert np.linalg.norm(g - want) / np.linalg.norm(want) < 1e-4


def test_oracle_stub_reproduces_reference_render_fixture_shapes():
    """The fixture's structure: render()'s key set for train (7 images) and debug (11)."""
    d = np.load(os.path.join(GOLD, "render.npz"), allow_pickle=False)
    base = ["alpha", "depth", "diffuse_color", "normal", "normal_ref", "render", "specular_color"]
    assert [str(k) for k in d["black/keys"]] == base
    assert [str(k) for k in d["white_debug/keys"]] == sorted(base + ["albedo", "metalness", "roughness", "sky_color"])
    H, W = int(d["H"]), int(d["W"])
    for k in base:
        assert d[f"black/out/{k}"].shape == (3, H, W), k
