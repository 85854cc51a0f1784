"""CPU: rotation of the environment SH (gsr/shrot.py, the relight sequence of
relit_novel_view.py:131-152).  Pinned through the reference-generated eval_sh goldens
(tests/golden/eval_sh.npz) by the rotated-direction identity
eval_sh(rot_R(c), R d) = eval_sh(c, d); spaudiopy's own Euler/sign convention is parity
unpinned (the package is absent)."""
import math
import os

import numpy as np
import pytest
import torch

from helpers import rel_l2

GOLD = os.path.join(os.path.dirname(__file__), "golden", "eval_sh.npz")


def _rand_rotation(seed):
    q = np.random.default_rng(seed).normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


@pytest.mark.parametrize("deg", [1, 2, 3, 4])
@pytest.mark.parametrize("which", ["y30", "y_end", "random"])
def test_rotated_lighting_equals_golden_at_rotated_directions(deg, which):
    from gsr import shrot, train
    g = np.load(GOLD)
    sh, dirs, out = g[f"sh{deg}"], g[f"dirs{deg}"], g[f"out{deg}"]   # sh [N,3,K], out [N,3]
    R = {"y30": shrot.rotation_y(math.pi / 6), "y_end": shrot.rotation_y(shrot.REF_ANGLE_END),
         "random": _rand_rotation(deg)}[which]
    c = torch.tensor(sh).transpose(1, 2)                              # [N,K,3]
    c_rot = shrot.rotate_sh(c.double(), R)
    d_rot = torch.tensor(dirs @ R.T)                                  # R d
    B = train.sh_basis(deg, d_rot.double())                           # [N,K]
    got = torch.einsum("nk,nkc->nc", B, c_rot).numpy()
    assert rel_l2(got, out) < 2e-6


def test_rotation_is_orthogonal_and_composes():
    from gsr import shrot
    a, b = 0.7, -1.9
    Ma, Mb = shrot.sh_rotation(4, shrot.rotation_y(a)), shrot.sh_rotation(4, shrot.rotation_y(b))
    Mab = shrot.sh_rotation(4, shrot.rotation_y(a + b))
    assert np.allclose(Ma @ Mb, Mab, atol=1e-10)
    assert np.allclose(Ma @ Ma.T, np.eye(25), atol=1e-10)
    assert np.allclose(shrot.sh_rotation(4, np.eye(3)), np.eye(25), atol=1e-12)
    # band 0 is invariant
    assert abs(Ma[0, 0] - 1.0) < 1e-12


def test_reference_angles():
    from gsr import shrot
    a = shrot.reference_angles()
    assert a.shape == (30,) and a[0] == 0.0 and abs(a[-1] - 6.28) < 1e-12
    seq = shrot.rotated_sequence(torch.randn(25, 3))
    assert len(seq) == 30 and all(s.shape == (25, 3) for s in seq)
