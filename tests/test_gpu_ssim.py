"""GPU: the fused SSIM (gsr_ssim.hip) against the reference's conv2d formulation
(utils/loss_utils.py:53-96, restated in test_train_cpu.ssim_conv2d) -- value and dL/dimg1,
with and without masks, ragged sizes, 1080p.  fp32: relative tolerance 1e-5 on the value,
1e-4 (relative L2) on the gradient (different summation orders)."""
import pytest
import torch

from helpers import rel_l2
from test_train_cpu import ssim_conv2d

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape,mask_kind", [((3, 97, 131), None), ((3, 64, 64), "one"), ((3, 75, 200), "full"),
                                             ((1, 40, 33), "one"), ((3, 1080, 1920), "one")])
def test_fused_ssim_matches_conv2d(shape, mask_kind):
    from gsr import train
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(5)
    C, H, W = shape
    base = torch.rand(shape, generator=g)
    a = (base + 0.1 * torch.randn(shape, generator=g)).to(dev)
    b = base.to(dev)
    if mask_kind is None:
        mask = None
    else:
        m = (torch.rand((1, H, W), generator=g) > 0.2).float()
        mask = m.expand(C, H, W).to(dev) if mask_kind == "one" else (torch.rand(shape, generator=g) > 0.3).float().to(dev)
    a1 = a.clone().requires_grad_(True)
    a2 = a.clone().requires_grad_(True)
    v1 = train.ssim(a1, b, mask)
    v2 = ssim_conv2d(a2, b, mask)
    (3.0 * v1).backward()
    (3.0 * v2).backward()
    torch.cuda.synchronize()
    f1, f2 = float(v1.detach()), float(v2.detach())
    assert abs(f1 - f2) <= 1e-5 * abs(f2) + 1e-7, (f1, f2)
    e = rel_l2(a1.grad.cpu().numpy(), a2.grad.cpu().numpy())
    assert e < 1e-4, e


def test_fused_ssim_empty_mask_is_one():
    from gsr import train
    a = torch.rand(3, 20, 20, device="cuda")
    assert float(train.ssim(a, a * 0.5, torch.zeros(3, 20, 20, device="cuda"))) == 1.0


@pytest.mark.parametrize("H,W,empty_sky", [(64, 96, False), (1080, 1920, False), (40, 40, True)])
def test_fused_view_loss_matches_torch(H, W, empty_sky):
    """train.py:77-99's loss: the fused pointwise kernels + fused SSIM against the same
    terms composed from PyTorch ops (train.view_loss_torch), value and the five gradients."""
    from gsr import train
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(9)
    names = ["render", "diffuse_color", "specular_color", "normal", "normal_ref"]
    base = {k: torch.rand(3, H, W, generator=g) for k in names}
    base["normal"] = base["normal"] * 2 - 1
    gt = torch.rand(3, H, W, generator=g).to(dev)
    sky = (torch.rand(1, H, W, generator=g) > 0.3).float()
    if empty_sky:
        sky.fill_(1.0)  # no non-sky pixel: the sky-BRDF L1s are 0 (the reference's early return)
    occ = (torch.rand(1, H, W, generator=g) > 0.1).float()
    sky3, occ3 = sky.expand(3, H, W).to(dev), occ.expand(3, H, W).to(dev)
    a = {k: v.to(dev).requires_grad_(True) for k, v in base.items()}
    b = {k: v.to(dev).requires_grad_(True) for k, v in base.items()}
    la = train.view_loss(a, gt, sky3, occ3)
    lb = train.view_loss_torch(b, gt, sky3, occ3)
    (2.0 * la).backward()
    (2.0 * lb).backward()
    torch.cuda.synchronize()
    fa, fb = float(la.detach()), float(lb.detach())
    assert abs(fa - fb) <= 1e-5 * abs(fb) + 1e-7, (fa, fb)
    for k in names:
        e = rel_l2(a[k].grad.cpu().numpy(), b[k].grad.cpu().numpy())
        assert e < 1e-5 or (b[k].grad.abs().max() == 0 and a[k].grad.abs().max() == 0), (k, e)


@pytest.mark.parametrize("H,W,case", [(64, 96, "plain"), (1080, 1920, "plain"), (40, 40, "empty_occ"),
                                      (33, 47, "empty_sky")])
def test_fused_objective_matches_scalar_tail(H, W, case):
    """The objective's scalar tail on the device (gsr_view_objective) and the SSIM gradient
    added onto the pointwise one against the same kernels with the tail in PyTorch
    (train.view_loss_unfused): value and gradients to 1e-6, including an empty occluder mask
    (SSIM 1, no reconstruction gradient) and no non-sky pixel."""
    from gsr import train
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(21)
    names = ["render", "diffuse_color", "specular_color", "normal", "normal_ref"]
    base = {k: torch.rand(3, H, W, generator=g) for k in names}
    gt = torch.rand(3, H, W, generator=g).to(dev)
    sky = (torch.rand(H, W, generator=g) > 0.3).float()
    occ = (torch.rand(H, W, generator=g) > 0.1).float()
    if case == "empty_occ":
        occ.zero_()
    if case == "empty_sky":
        sky.fill_(1.0)
    sky, occ = sky.to(dev), occ.to(dev)
    a = {k: v.to(dev).requires_grad_(True) for k, v in base.items()}
    b = {k: v.to(dev).requires_grad_(True) for k, v in base.items()}
    la = train.view_loss(a, gt, sky, occ)
    lb = train.view_loss_unfused(b, gt, sky, occ)
    assert la.dim() == 0 and la.dtype == torch.float32
    (3.0 * la).backward()
    (3.0 * lb).backward()
    torch.cuda.synchronize()
    fa, fb = float(la.detach()), float(lb.detach())
    assert abs(fa - fb) <= 1e-6 * abs(fb) + 1e-7, (fa, fb)
    for k in names:
        ga, gb = a[k].grad, b[k].grad
        if float(gb.abs().max()) == 0:
            assert float(ga.abs().max()) == 0, k
            continue
        assert rel_l2(ga.cpu().numpy(), gb.cpu().numpy()) < 1e-6, k


@pytest.mark.parametrize("H,W,occ_kind", [(97, 131, "rand"), (1080, 1920, "rand"), (64, 80, "empty")])
def test_ssim_l1_backward_matches_two_pass(H, W, occ_kind):
    """gsr_ssim_l1_backward (the image gradient's L1 term made inside the SSIM backward) against
    the two-pass path it replaces: gsr_view_loss_backward's d_img, then gsr_ssim_backward with
    accumulate.  Same two roundings per value (no contraction across them): equal up to the
    SSIM term's own fused multiply-add, checked at 1e-6 relative per value."""
    import ctypes as C
    from gsr import _lib, train
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(7)
    img = torch.rand(3, H, W, device=dev, generator=g)
    gt = (img + 0.05 * torch.randn(3, H, W, device=dev, generator=g)).clamp(0, 1)
    gt[:, : H // 4] = img[:, : H // 4]  # exact ties: sign 0 in the L1 term
    planes = [torch.rand(3, H, W, device=dev, generator=g) for _ in range(4)]  # diff, spec, nrm, nref
    sky = (torch.rand(H, W, device=dev, generator=g) > 0.3).float()
    occ = torch.zeros(H, W, device=dev) if occ_kind == "empty" else (torch.rand(H, W, device=dev, generator=g) > 0.2).float()
    L = _lib.lib()
    st = _lib.stream_of(dev)
    win = (C.c_float * 11)(*train.gaussian_1d(11).tolist())
    nss = int(L.gsr_ssim_partials(3, H, W))
    parts = torch.empty(2 * nss, device=dev)
    dmaps = torch.empty(3, 3, H, W, device=dev)
    _lib.check(L.gsr_ssim_forward(3, H, W, img.data_ptr(), gt.data_ptr(), occ.data_ptr(), 0, win, parts.data_ptr(),
                                  dmaps.data_ptr(), st), "gsr_ssim_forward")
    coef = torch.tensor([0.37, 0.11, -0.02, -0.61], device=dev)  # (k_img, k_brdf, k_normal, k_ssim)
    ts = [img, gt, *planes, sky, occ]
    two = torch.empty_like(img)
    _lib.check(L.gsr_view_loss_backward(H * W, *[t.data_ptr() for t in ts], coef.data_ptr(), two.data_ptr(), None, None,
                                        None, None, st), "gsr_view_loss_backward")
    _lib.check(L.gsr_ssim_backward(3, H, W, img.data_ptr(), gt.data_ptr(), dmaps.data_ptr(), coef.data_ptr() + 12, win,
                                   two.data_ptr(), 1, st), "gsr_ssim_backward")
    one = torch.full_like(img, float("nan"))
    _lib.check(L.gsr_ssim_l1_backward(3, H, W, img.data_ptr(), gt.data_ptr(), dmaps.data_ptr(), coef.data_ptr() + 12,
                                      win, occ.data_ptr(), coef.data_ptr(), one.data_ptr(), st), "gsr_ssim_l1_backward")
    torch.cuda.synchronize()
    assert torch.isfinite(one).all()
    d = (one - two).abs()
    assert float(d.max()) <= 1e-6 * float(two.abs().max()) + 1e-12, float(d.max())
    if occ_kind == "empty":  # no mask: no L1 term and a zero SSIM gradient
        assert float(one.abs().max()) == 0.0
