"""Geometry cache across same-geometry rasterizer calls (render()'s 6-10
calls per view): cached calls must be bit-identical to full calls, in the forward and in
the backward, and any change of a geometry input must miss."""
import math

import pytest
import torch

from helpers import make_case

pytestmark = pytest.mark.gpu


def _setup(P=4000, W=160, H=96, seed=0):
    import diff_gaussian_rasterization as dgr
    cam, gs = make_case(P=P, W=W, H=H, sh_degree=0, seed=seed, camera="orbit")
    dev = torch.device("cuda")
    g = {k: v.to(dev) for k, v in gs.items()}

    def settings(bg):
        return dgr.GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
            bg=torch.tensor(bg, dtype=torch.float32, device=dev), scale_modifier=1.0,
            viewmatrix=cam.world_view_transform.to(dev), projmatrix=cam.full_proj_transform.to(dev), sh_degree=0,
            campos=cam.camera_center.to(dev), prefiltered=False)
    return dgr, g, settings


def _render_calls(dgr, g, settings, colors_list, bgs, cached):
    """Like render(): one set of geometry tensors, several colour sets; returns images and
    the gradients of sum(w_k * image_k)."""
    cache = dgr.geometry_cache(cached)
    means3D = g["means3D"].clone().requires_grad_(True)
    opac = g["opacities"].clone().requires_grad_(True)
    scales = g["scales"].clone().requires_grad_(True)
    rots = g["rotations"].clone().requires_grad_(True)
    means2D = torch.zeros_like(means3D, requires_grad=True)
    # one settings object per call, as render() builds them; matrices are the same tensors
    base = settings(bgs[0])
    cols = [c.clone().requires_grad_(True) for c in colors_list]
    imgs, radii = [], []
    for c, bg in zip(cols, bgs):
        s = base._replace(bg=torch.tensor(bg, dtype=torch.float32, device="cuda"))
        img, r = dgr.GaussianRasterizer(s)(means3D=means3D, means2D=means2D, opacities=opac, colors_precomp=c,
                                           scales=scales, rotations=rots)
        imgs.append(img)
        radii.append(r)
    gen = torch.Generator(device="cuda").manual_seed(4)
    loss = sum((torch.randn(img.shape, device="cuda", generator=gen) * img).sum() for img in imgs)
    loss.backward()
    grads = [means3D.grad, opac.grad, scales.grad, rots.grad, means2D.grad] + [c.grad for c in cols]
    stats = (cache.hits, cache.misses)
    dgr.geometry_cache(True)
    return imgs, radii, grads, stats


def test_cached_calls_match_full_calls_bitwise():
    dgr, g, settings = _setup()
    gen = torch.Generator(device="cuda").manual_seed(2)
    colors = [torch.rand(g["means3D"].shape[0], 3, device="cuda", generator=gen) for _ in range(4)]
    colors.append(torch.ones_like(colors[0]))  # the alpha call
    bgs = [(0.0, 0.0, 0.0), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0), (0.3, 0.2, 0.1), (0.0, 0.0, 0.0)]
    imgs_c, radii_c, grads_c, (hits, misses) = _render_calls(dgr, g, settings, colors, bgs, cached=True)
    imgs_f, radii_f, grads_f, (hits_f, _) = _render_calls(dgr, g, settings, colors, bgs, cached=False)
    assert (hits, misses) == (4, 1) and hits_f == 0
    for a, b in zip(imgs_c, imgs_f):
        assert torch.equal(a, b)
    for a, b in zip(radii_c, radii_f):
        assert torch.equal(a, b)
    # the backward per call is the same kernel on the same buffers contents; summation
    # order over calls is the same, but the render backward's atomics make bits differ run
    # to run, so compare to the tolerance of the parity tests
    for a, b in zip(grads_c, grads_f):
        d = torch.linalg.norm((a - b).double()) / torch.linalg.norm(b.double()).clamp_min(1e-30)
        assert d < 1e-5, d


def test_geometry_change_misses():
    import diff_gaussian_rasterization as dgr
    _, g, settings = _setup(P=2000, W=64, H=64)
    cache = dgr.geometry_cache(True)
    s = settings((0.0, 0.0, 0.0))
    col = torch.rand(g["means3D"].shape[0], 3, device="cuda")
    means3D = g["means3D"].clone()
    run = lambda **kw: dgr.GaussianRasterizer(s)(**{**dict(means3D=means3D, means2D=torch.zeros_like(means3D),
                                                            opacities=g["opacities"], colors_precomp=col,
                                                            scales=g["scales"], rotations=g["rotations"]), **kw})
    run()
    run()
    assert (cache.hits, cache.misses) == (1, 1)
    means3D.add_(0.0)  # in-place update (optimizer step): version bump
    run()
    assert cache.misses == 2
    run(opacities=g["opacities"].clone())  # a new tensor
    assert cache.misses == 3
    s2 = s._replace(scale_modifier=1.5)
    dgr.GaussianRasterizer(s2)(means3D=means3D, means2D=torch.zeros_like(means3D), opacities=g["opacities"],
                              colors_precomp=col, scales=g["scales"], rotations=g["rotations"])
    assert cache.misses == 4
    # SH colours are never served from the cache
    hits = cache.hits
    dgr.GaussianRasterizer(s)(means3D=means3D, means2D=torch.zeros_like(means3D), opacities=g["opacities"],
                              shs=torch.zeros(means3D.shape[0], 1, 3, device="cuda"), scales=g["scales"],
                              rotations=g["rotations"])
    assert cache.hits == hits


def test_cache_is_keyed_on_the_stream():
    """a hit reuses buffers ordered only on the miss call's stream, so the same
    geometry rendered on another HIP stream must miss (and still be bit-identical)."""
    dgr, g, settings = _setup(P=3000)
    cache = dgr.geometry_cache(True)
    s = settings((0.0, 0.0, 0.0))
    gen = torch.Generator(device="cuda").manual_seed(9)
    c1 = torch.rand(g["means3D"].shape[0], 3, device="cuda", generator=gen)
    call = lambda c: dgr.GaussianRasterizer(s)(means3D=g["means3D"], means2D=torch.zeros_like(g["means3D"]),
                                               opacities=g["opacities"], colors_precomp=c, scales=g["scales"],
                                               rotations=g["rotations"])[0]
    a = call(c1)
    m0, h0 = cache.misses, cache.hits
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        b = call(c1)
    torch.cuda.current_stream().wait_stream(side)
    assert cache.misses == m0 + 1 and cache.hits == h0
    c = call(c1)  # back on the main stream: the side stream's entry is not reused either
    assert cache.misses == m0 + 2
    d = call(c1)  # same stream again: hit
    assert cache.hits == h0 + 1
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(a, c) and torch.equal(a, d)


def test_deterministic_backward_after_cached_forward():
    """deterministic mode switched on between cached forwards (gsr_forward_reuse)
    and their backward: the gather needs every call's rects and depth keys, which the reuse
    path copies whatever the mode at forward time.  The gradients match the atomic backward
    of the same calls (1e-5, summation order)."""
    from gsr import _lib
    dgr, g, settings = _setup(P=3000, W=128, H=96)
    gen = torch.Generator(device="cuda").manual_seed(5)
    colors = [torch.rand(g["means3D"].shape[0], 3, device="cuda", generator=gen) for _ in range(3)]
    bgs = [(0.0, 0.0, 0.0)] * 3

    def run(det_at_backward):
        dgr.geometry_cache(True)
        means3D = g["means3D"].clone().requires_grad_(True)
        cols = [c.clone().requires_grad_(True) for c in colors]
        s = settings(bgs[0])
        imgs = [dgr.GaussianRasterizer(s)(means3D=means3D, means2D=torch.zeros_like(means3D), opacities=g["opacities"],
                                          colors_precomp=c, scales=g["scales"], rotations=g["rotations"])[0]
                for c in cols]
        w = torch.Generator(device="cuda").manual_seed(6)
        loss = sum((torch.randn(i.shape, device="cuda", generator=w) * i).sum() for i in imgs)
        _lib.set_deterministic(det_at_backward)
        try:
            loss.backward()
            torch.cuda.synchronize()
        finally:
            _lib.set_deterministic(False)
        return [means3D.grad.cpu()] + [c.grad.cpu() for c in cols]

    a, d = run(False), run(True)
    for x, y in zip(a, d):
        assert torch.isfinite(y).all()
        e = torch.linalg.norm((x - y).double()) / torch.linalg.norm(x.double()).clamp_min(1e-30)
        assert e < 1e-5, e
