"""Rotation of real spherical-harmonic lighting coefficients (relit_novel_view.py:131-152).

The reference relights a novel view under its environment SH rotated about the vertical
axis, 30 angles over [0, 6.28] (``np.interp(np.linspace(0, 1, 30), [0, 1], [0, 3.14*2])``,
:131-136), by ``spaudiopy.sph.rotate_sh(F, 0, angle, 0, 'real')`` (:139-140), then renders
with ``fix_sky=True`` and a zero sky SH (:147-149).

spaudiopy is absent here (and unpinned in environment.yml), so its Euler-angle and sign
conventions are **parity unpinned**.  This module rotates in the basis the shade actually
evaluates, eval_sh (utils/sh_utils.py:81-151), so the rotated lighting is exactly the
original lighting turned by R:

    eval_sh(rotate_sh(c, R), d) == eval_sh(c, R^T d)        for every unit d,

which tests/test_shrot.py checks against the reference-generated eval_sh golden vectors.
Each band l maps onto itself under rotation, so the rotation is block diagonal with one
(2l+1)x(2l+1) block per band; a block is solved in float64 from the basis at 4(2l+1)
directions (exact up to rounding: the band is a rotation-invariant space).  The matrices
are tiny (25x25 at degree 4) and computed on the host once per angle.
"""
from __future__ import annotations

import math
from typing import Dict, List, Tuple

import numpy as np
import torch

REF_STEPS, REF_ANGLE_END = 30, 3.14 * 2  # relit_novel_view.py:131-136


def reference_angles(steps: int = REF_STEPS) -> np.ndarray:
    """The reference's sun angles: np.interp(np.linspace(0, 1, steps), [0, 1], [0, 3.14*2])."""
    return np.interp(np.linspace(0, 1, steps), [0, 1], [0.0, REF_ANGLE_END])


def rotation_y(angle: float) -> np.ndarray:
    """Right-handed rotation by ``angle`` about +y (acting on column vectors)."""
    c, s = math.cos(angle), math.sin(angle)
    return np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])


def _basis64(deg: int, d: np.ndarray) -> np.ndarray:
    from .train import sh_basis
    return sh_basis(deg, torch.from_numpy(d)).numpy()


def _fib_dirs(n: int) -> np.ndarray:
    """n well-spread unit directions (Fibonacci sphere), float64."""
    i = np.arange(n) + 0.5
    z = 1.0 - 2.0 * i / n
    r = np.sqrt(np.maximum(0.0, 1.0 - z * z))
    phi = math.pi * (3.0 - math.sqrt(5.0)) * i
    return np.stack([r * np.cos(phi), r * np.sin(phi), z], 1)


_CACHE: Dict[Tuple[int, bytes], np.ndarray] = {}


def sh_rotation(deg: int, R: np.ndarray) -> np.ndarray:
    """[K,K] float64 (K = (deg+1)^2), block diagonal by band: rotated = M @ coeffs, with
    eval_sh(M @ c, d) = eval_sh(c, R^T d)."""
    R = np.asarray(R, np.float64)
    key = (deg, R.tobytes())
    M = _CACHE.get(key)
    if M is not None:
        return M
    K = (deg + 1) ** 2
    d = _fib_dirs(8 * K)
    B = _basis64(deg, d)                 # Y(d)        [N,K]
    Bt = _basis64(deg, d @ R)            # Y(R^T d)    [N,K]  (rows d_i^T R = (R^T d_i)^T)
    M = np.zeros((K, K))
    for l in range(deg + 1):
        a, b = l * l, (l + 1) * (l + 1)
        # f'(d) = sum_m c_m Y_m(R^T d) = sum_m' c'_m' Y_m'(d)  =>  Y_l(R^T d) = Y_l(d) @ X,  c' = X @ c
        X, *_ = np.linalg.lstsq(B[:, a:b], Bt[:, a:b], rcond=None)
        M[a:b, a:b] = X
    _CACHE[key] = M
    return M


def rotate_sh(coeffs: torch.Tensor, R: np.ndarray) -> torch.Tensor:
    """coeffs [..., K, C] (the envlight base layout [25, 3]) rotated by R, same dtype/device."""
    K = coeffs.shape[-2]
    deg = int(round(math.sqrt(K))) - 1
    if (deg + 1) ** 2 != K:
        raise ValueError(f"rotate_sh: {K} coefficients is not a full SH degree")
    M = torch.from_numpy(sh_rotation(deg, R)).to(device=coeffs.device, dtype=torch.float64)
    return (M @ coeffs.double()).to(coeffs.dtype)


def rotated_sequence(base: torch.Tensor, steps: int = REF_STEPS) -> List[torch.Tensor]:
    """The reference's relight sequence: ``base`` rotated about y by each reference angle."""
    return [rotate_sh(base, rotation_y(float(a))) for a in reference_angles(steps)]
