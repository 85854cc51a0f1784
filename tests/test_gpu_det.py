"""Deterministic backward mode and the GSR_DEBUG build.

* Deterministic mode (gsr_set_deterministic): the tile passes write each (tile, Gaussian)
  pair's partial sums to a per-instance row and one pass sums each Gaussian's rows in a
  fixed order, instead of float atomics.  Its gradients must be bit-identical run to run and
  within 1e-6 relative L2 of the atomic path (the same partial sums, added in a different
  order), for the 3-channel and the multi-channel backward.
* The invariant checker (gsr_check_buffers; run after every forward by the GSR_DEBUG build
  lib/debug/libgsr.so) must pass on real forwards and name a corrupted list.
* The GSR_DEBUG build must pass the forward/backward parity suite (in a child process, since
  one process loads one libgsr)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from helpers import make_case, rel_l2
from test_gpu_rasterizer import CASES, _view, mutate, run_gpu

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DET_CASES = [c for c in CASES if c["name"] in ("cfg1_small_sh0", "sh3_orbit_bg", "dense_small", "half_outside",
                                                "opaque_stack", "heavy_tiles")]


def _backward(case, det, surv=True):
    from diff_gaussian_rasterization import _C
    from gsr import _lib
    cam, gs = make_case(P=case["P"], W=case["W"], H=case["H"], sh_degree=case.get("sh_degree", 0),
                        camera=case.get("camera", "identity"))
    gs = mutate(gs, case.get("mutate"))
    kw = dict(mode=case["mode"], bg=case.get("bg", (0.0, 0.0, 0.0)), sh_degree=case.get("sh_degree", 0))
    _lib.set_deterministic(det)
    _lib.set_survivor_lists(surv)
    try:
        assert _lib.deterministic() == det and _lib.survivor_lists() == surv
        st = run_gpu(cam, gs, **kw)
        dout = torch.randn(3, cam.image_height, cam.image_width, generator=torch.Generator().manual_seed(1))
        grads = _C.rasterize_gaussians_backward(
            st["bg"], st["means"], st["radii"], st["colors"], st["scales"], st["rots"], 1.0, st["cov3"], st["vm"],
            st["pm"], cam.tanfovx, cam.tanfovy, dout.cuda(), st["sh"], kw["sh_degree"], st["cp"], st["geom"],
            st["R"], st["binb"], st["img"])
        torch.cuda.synchronize()
    finally:
        _lib.set_deterministic(False)
        _lib.set_survivor_lists(True)
    return [g.detach().cpu() for g in grads]


@pytest.mark.parametrize("case", DET_CASES, ids=[c["name"] for c in DET_CASES])
def test_deterministic_backward(case):
    atomic = _backward(case, False)
    d1 = _backward(case, True)
    d2 = _backward(case, True)
    for k, (a, x, y) in enumerate(zip(atomic, d1, d2)):
        assert torch.equal(x, y), f"gradient {k} differs between two deterministic runs"
        if a.numel() == 0 or not a.abs().max() > 0:
            assert x.numel() == a.numel() and (x.numel() == 0 or x.abs().max() == 0), k
            continue
        e = rel_l2(x.numpy(), a.numpy())
        assert e <= 1e-6, (k, e)


@pytest.mark.parametrize("case", DET_CASES, ids=[c["name"] for c in DET_CASES])
def test_survivor_lists_change_nothing(case):
    """The backward over the forward's survivor lists evaluates the same (Gaussian, quadrant)
    pairs in the same order as the one that filters the super-tile lists again: in
    deterministic mode (no atomics) every gradient is bit-identical."""
    with_lists = _backward(case, True, surv=True)
    without = _backward(case, True, surv=False)
    for k, (x, y) in enumerate(zip(with_lists, without)):
        assert torch.equal(x, y), f"gradient {k} differs with the survivor lists"


def test_deterministic_multichannel():
    """render_channels' 14-channel composite backward: deterministic runs bit-identical, and
    within 1e-6 of the atomic composite."""
    import diff_gaussian_rasterization as dgr
    from gsr import _lib
    from test_gpu_channels import _colour_sets, _multi, _setup
    _, g, s = _setup(P=6000, W=150, H=100)
    ks = [3, 3, 3, 1, 3, 1]
    cols = _colour_sets(6000, ks)
    bgs = [torch.rand(k, device="cuda") for k in ks]
    gen = torch.Generator(device="cuda").manual_seed(4)
    weights = [torch.randn(k, 100, 150, device="cuda", generator=gen) for k in ks]

    def run(det, surv=True):
        _lib.set_deterministic(det)
        _lib.set_survivor_lists(surv)
        try:
            _, _, grads, cgrads = _multi(dgr, g, s, cols, bgs, weights)
            torch.cuda.synchronize()
        finally:
            _lib.set_deterministic(False)
            _lib.set_survivor_lists(True)
        return [t.detach().cpu() for t in grads + cgrads]

    a, d1, d2, d3 = run(False), run(True), run(True), run(True, surv=False)
    for k, (x, y, z, w) in enumerate(zip(a, d1, d2, d3)):
        assert torch.equal(y, z), k
        assert torch.equal(y, w), f"{k}: the survivor lists changed a deterministic gradient"
        if x.abs().max() > 0:
            assert rel_l2(y.numpy(), x.numpy()) <= 1e-6, (k, rel_l2(y.numpy(), x.numpy()))


def test_check_buffers_accepts_and_rejects():
    """gsr_check_buffers materialises the reference's lists from the super-tile entries and
    verifies them; a corrupted entry must be named."""
    from gsr import _lib
    case = next(c for c in CASES if c["name"] == "dense_small")
    cam, gs = make_case(P=case["P"], W=case["W"], H=case["H"])
    st = run_gpu(cam, gs, mode="colors")
    P, R, W, H = case["P"], st["R"], case["W"], case["H"]
    _lib.check_buffers(P, R, W, H, st["radii"], st["geom"], st["binb"], st["img"])
    L = _lib.layout(P, R, W, H)
    NS = ((W + 15) // 16 + 7) // 8 * (((H + 15) // 16 + 3) // 4)
    st_ranges = _view(st["binb"], L.bin_st_ranges, 2 * NS, torch.int32).view(NS, 2).cpu().numpy()
    S = int(st_ranges[:, 1].max())
    ent = _view(st["binb"], L.bin_entries, 2 * S, torch.int32).view(S, 2)  # aliases the binning buffer
    k = int(np.argmax(st_ranges[:, 1] - st_ranges[:, 0]))
    x = int(st_ranges[k, 0])
    saved = ent[x + 1].clone()
    ent[x + 1] = ent[x]  # a duplicated entry: its tiles list one Gaussian twice
    with pytest.raises(RuntimeError, match="order"):
        _lib.check_buffers(P, R, W, H, st["radii"], st["geom"], st["binb"], st["img"])
    ent[x + 1] = saved
    _lib.check_buffers(P, R, W, H, st["radii"], st["geom"], st["binb"], st["img"])
    saved = ent[x].clone()
    ent[x, 1] = P  # an id past the end
    with pytest.raises(RuntimeError, match="id >= P"):
        _lib.check_buffers(P, R, W, H, st["radii"], st["geom"], st["binb"], st["img"])
    ent[x] = saved


def test_debug_build_parity_suite():
    """The GSR_DEBUG library (its forward verifies every tile list on the device) passes the
    forward/backward parity cases and the speculative-binning overflow test."""
    from gsr import _lib
    assert os.path.exists(_lib.DEBUG_LIB_PATH), "lib/debug/libgsr.so not built (__graft_entry__.build())"
    env = dict(os.environ, GSR_LIB_PATH=_lib.DEBUG_LIB_PATH)
    probe = subprocess.run([sys.executable, "-c", "import sys; sys.path[:0] = [sys.argv[1]]; from gsr import _lib; "
                            "assert _lib.debug_build(); print('debug build')",
                            os.path.join(ROOT, "relightable3dgaussians-w_amd")], env=env, capture_output=True,
                           text=True, timeout=120)
    assert probe.returncode == 0 and "debug build" in probe.stdout, probe.stderr[-2000:]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_gpu_rasterizer.py"), "-k",
                        "forward_parity or backward_parity or speculative or empty"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
