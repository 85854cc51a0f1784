"""Survivor lists on frames large enough to use them.

The forward's whole-tile units store each tile's survivors and the backward walks them; tiles
the forward splits into quadrant units (each band's 128 lightest, and heavy ones) and tiles
with more than SURV_CAP survivors keep the super-tile path.  The small parity cases of
test_gpu_rasterizer have bands of fewer than 128 tiles, so every tile there is split and none
has a list: this file renders 1024 x 768 (384 tiles per band) with a faint, wide clump over a
few tiles so that both kinds of tile occur, and checks

* that lists are stored (most tiles) and that the clump's tiles overflowed SURV_CAP;
* the deterministic backward (no atomics) with lists against it without them: bit-identical
  gradients (the same evaluations in the same order);
* the atomic backward with lists against the deterministic one without them: 1e-6."""
import numpy as np
import pytest
import torch

from helpers import make_case, rel_l2
from test_gpu_rasterizer import _view, run_gpu

pytestmark = pytest.mark.gpu

W, H = 1024, 768
SURV_NONE = 0xFFFFFFFF


def _scene():
    cam, gs = make_case(P=60000, W=W, H=H, sh_degree=1)
    g = torch.Generator().manual_seed(3)
    # a clump: 2500 faint, wide copies of one Gaussian near the image centre (alpha ~0.006: a
    # pixel saturates only after ~1500 of them, past SURV_CAP), jittered along its ray
    means = gs["means3D"]
    d = means[:, :2] / means[:, 2:3]
    k = int(torch.argmin((d ** 2).sum(1)))
    n = 2500
    c = {key: v[k:k + 1].repeat(n, *([1] * (v.dim() - 1))).clone() for key, v in gs.items()}
    c["means3D"] = c["means3D"] * (1.0 + 0.05 * torch.rand(n, 1, generator=g))
    c["means3D"][:, :2] += 0.02 * torch.randn(n, 2, generator=g)
    c["scales"] = c["scales"] * 2.0
    c["opacities"] = torch.full_like(c["opacities"], 0.006)
    gs = {key: torch.cat([gs[key], c[key]]) for key in gs}
    return cam, gs


def _grads(cam, gs, det, surv):
    from diff_gaussian_rasterization import _C
    from gsr import _lib
    _lib.set_deterministic(det)
    _lib.set_survivor_lists(surv)
    try:
        st = run_gpu(cam, gs, mode="sh", sh_degree=1)
        dout = torch.randn(3, H, W, generator=torch.Generator().manual_seed(1))
        grads = _C.rasterize_gaussians_backward(
            st["bg"], st["means"], st["radii"], st["colors"], st["scales"], st["rots"], 1.0, st["cov3"], st["vm"],
            st["pm"], cam.tanfovx, cam.tanfovy, dout.cuda(), st["sh"], 1, st["cp"], st["geom"], st["R"],
            st["binb"], st["img"])
        torch.cuda.synchronize()
        P = gs["means3D"].shape[0]
        L = _lib.layout(P, st["R"], W, H)
        T = ((W + 15) // 16) * ((H + 15) // 16)
        sn = _view(st["img"], L.img_surv_n, T, torch.int32).cpu().numpy().view(np.uint32).copy()
        nc = st["rec"][:, :2].copy()  # the Gaussians' screen centres (pixels)
    finally:
        _lib.set_deterministic(False)
        _lib.set_survivor_lists(True)
    return [x.detach().cpu() for x in grads], sn, nc, L.surv_cap


def test_survivor_lists_at_size():
    cam, gs = _scene()
    g_det_l, sn, nc, cap = _grads(cam, gs, True, True)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    assert cap > 0
    lst = sn != SURV_NONE
    assert lst.mean() > 0.5, f"only {lst.mean():.2f} of the tiles stored a list"
    assert (sn[lst] <= cap).all()
    # the clump's centre tile reaches SURV_CAP before it saturates (~1500 of its 2500 faint
    # Gaussians blend at every pixel there): no list
    x, y = nc[-1]
    t = int(y // 16) * gx + int(x // 16)
    assert not lst[t], f"the clump's tile {t} stored a list of {sn[t]} (cap {cap})"
    g_det_n, sn2, _, _ = _grads(cam, gs, True, False)
    assert (sn2 == SURV_NONE).all(), "lists stored although switched off"
    for k, (x, y) in enumerate(zip(g_det_l, g_det_n)):
        assert torch.equal(x, y), f"gradient {k} differs with the survivor lists"
    g_atomic, _, _, _ = _grads(cam, gs, False, True)
    for k, (x, y) in enumerate(zip(g_atomic, g_det_n)):
        if y.numel() and y.abs().max() > 0:
            assert rel_l2(x.numpy(), y.numpy()) <= 1e-6, (k, rel_l2(x.numpy(), y.numpy()))
