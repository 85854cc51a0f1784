"""Shared test helpers: scene builders and comparison utilities (test infrastructure)."""
import math

import numpy as np
import torch

from gsr import scenes


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32) if isinstance(t, torch.Tensor) else np.asarray(t, np.float32)


def make_case(P=2000, W=96, H=80, sh_degree=0, seed=0, fov_deg=60.0, camera="identity", opacity_hi=0.99,
              zrange=(2.0, 8.0), scale_mode="cfg1"):
    """Small deterministic scene; camera 'identity' (R=I, T=0) or 'orbit' (a rotated and
    translated camera looking at the cloud)."""
    fov = math.radians(fov_deg)
    cam = scenes.make_camera(W, H, fov, fov * H / W)
    gs = scenes.synthetic_gaussians(P, W, H, cam.tanfovx, cam.tanfovy, sh_degree, seed=seed, zrange=zrange,
                                    scale_mode=scale_mode)
    if opacity_hi != 0.99:
        gs["opacities"] = gs["opacities"].clamp(max=opacity_hi)
    if camera == "orbit":
        c = np.array([1.2, -0.8, -0.5])
        R, T = scenes.look_at_rotation(c, np.array([0.1, 0.0, 5.0]))
        cam = scenes.make_camera(W, H, fov, fov * H / W, R=R, T=T)
    return cam, gs


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def assert_close_rel(a, b, tol, name=""):
    e = rel_l2(a, b)
    assert e <= tol, f"{name}: rel L2 error {e:.3e} > {tol:.1e}"
    return e
