"""Views in flight on several HIP streams (bench.py's mini-batch step, the training step's
view streams): every call allocates its buffers on its own stream and syncs only that
stream, so concurrent views must give exactly the single-stream results -- images, radii
and the sorted binning bit for bit, gradients within the summation-order tolerance."""
import pytest
import torch

from helpers import make_case, rel_l2

pytestmark = pytest.mark.gpu


def _view(_C, cam, g, dout, dev):
    e = torch.empty(0, device=dev)
    bg = torch.zeros(3, device=dev)
    vm, pm, cp = cam.world_view_transform.to(dev), cam.full_proj_transform.to(dev), cam.camera_center.to(dev)
    R, color, radii, geom, binb, img = _C.rasterize_gaussians(
        bg, g["means3D"], e, g["opacities"], g["scales"], g["rotations"], 1.0, e, vm, pm, cam.tanfovx, cam.tanfovy,
        cam.image_height, cam.image_width, g["shs"], 3, cp, False)
    grads = _C.rasterize_gaussians_backward(bg, g["means3D"], radii, e, g["scales"], g["rotations"], 1.0, e, vm, pm,
                                            cam.tanfovx, cam.tanfovy, dout, g["shs"], 3, cp, geom, R, binb, img)
    return R, color, radii, grads


def test_concurrent_views_match_sequential():
    from diff_gaussian_rasterization import _C
    dev = torch.device("cuda")
    cases = []
    for k, camera in enumerate(("identity", "orbit", "identity", "orbit")):
        cam, gs = make_case(P=40000, W=320, H=200, sh_degree=3, seed=k, camera=camera)
        g = {n: v.to(dev) for n, v in gs.items()}
        dout = torch.randn(3, 200, 320, generator=torch.Generator().manual_seed(k)).to(dev)
        cases.append((cam, g, dout))
    ref = [_view(_C, cam, g, dout, dev) for cam, g, dout in cases]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    main = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(main)
    got = []
    for i, (cam, g, dout) in enumerate(cases):
        with torch.cuda.stream(streams[i % 2]):
            got.append(_view(_C, cam, g, dout, dev))
    for s in streams:
        main.wait_stream(s)
    torch.cuda.synchronize()
    for (R0, c0, r0, g0), (R1, c1, r1, g1) in zip(ref, got):
        assert R0 == R1
        assert torch.equal(r0, r1)
        assert torch.equal(c0, c1)
        for a, b in zip(g0, g1):
            if b.numel() and b.abs().max() > 0:
                assert rel_l2(a.cpu().numpy(), b.cpu().numpy()) < 1e-5
