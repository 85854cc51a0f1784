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
