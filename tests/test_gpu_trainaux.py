"""GPU: the training step's fused bookkeeping kernels (csrc/gsr_trainaux.hip) against the
PyTorch compositions they replace in gsr/train.py and gsr/dp.py (themselves pinned on the
CPU by tests/test_train_golden.py and tests/test_train_sky.py against the reference's
functions): the view regularisers and their gradients, the SH basis, the sky shell and its
gradients, the densification statistics.  fp32 sums over different orders: relative 1e-5;
the integer-valued counts and the elementwise results exact or within 1 ulp-scale bars
written per check."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pc(P, V, dev, seed=0, sky_frac=0.15):
    import types
    g = torch.Generator().manual_seed(seed)
    xyz = (torch.randn(P, 3, generator=g) * 3 + torch.tensor([0.0, 0.0, 6.0])).to(dev).requires_grad_(True)
    scaling = (torch.rand(P, 3, generator=g) * 0.2 + 1e-3).to(dev)
    scaling[::7, 1] = scaling[::7, 0]  # ties: torch.min's gradient goes to the first minimum
    scaling = scaling.requires_grad_(True)
    is_sky = (torch.rand(P, 1, generator=g) < sky_frac).to(dev)
    radii = [((torch.rand(P, generator=g) < 0.6) * torch.randint(1, 30, (P,), generator=g)).int().to(dev)
             for _ in range(V)]
    vms = torch.randn(V, 4, 4, generator=g).to(dev)
    env = (torch.randn(V, 25, 3, generator=g) * 0.3).to(dev).requires_grad_(True)
    dirs = (torch.rand(V, 10, 3, generator=g) * 2 - 1).to(dev)
    pc = types.SimpleNamespace(get_xyz=xyz, get_scaling=scaling, get_is_sky=is_sky)
    return pc, radii, vms, env, dirs


@pytest.mark.parametrize("tail", [True, False])
@pytest.mark.parametrize("P,V,depth_on", [(1000, 1, True), (70001, 4, True), (70001, 4, False), (4099, 8, True),
                                          (4099, 11, True)])  # 11: two launches of up to 8 views
def test_view_regularisers_fused_matches_torch(P, V, depth_on, tail):
    """The fused regularisers (per-Gaussian sums, and with ``tail`` the scalar tail and the
    envlight term in one workgroup) against the PyTorch composition: values and the xyz,
    scaling and environment-SH gradients."""
    from gsr import train
    pc, radii, vms, env, dirs = _pc(P, V, "cuda", seed=P + V)
    got = train.view_regularisers(pc, radii, vms, env, dirs, depth_on=depth_on, fused=True, tail_fused=tail)
    w = torch.randn(V, device="cuda")
    gg = torch.autograd.grad((got * w).sum(), [pc.get_xyz, pc.get_scaling, env], allow_unused=True)
    ref = train.view_regularisers(pc, torch.stack(radii), vms, env, dirs, depth_on=depth_on, fused=False)
    gr = torch.autograd.grad((ref * w).sum(), [pc.get_xyz, pc.get_scaling, env], allow_unused=True)
    assert torch.allclose(got, ref, rtol=1e-5, atol=1e-6), (got, ref)
    for name, a, b in zip(("xyz", "scaling", "env"), gg, gr):
        if b is None:
            assert a is None or float(a.abs().max()) == 0.0, name
            continue
        e = float((a - b).norm() / b.norm().clamp(min=1e-30))
        assert e < 1e-5, (name, e)


def test_view_regularisers_sums_exact_counts():
    """The per-view counts are exact integers and the sums match float64 references."""
    from gsr import _lib
    P, V = 50003, 3
    pc, radii, vms, env, dirs = _pc(P, V, "cuda", seed=9)
    from gsr.train import _FusedViewRegs
    c = vms[:, :, 2].contiguous()
    sums = _FusedViewRegs.apply(pc.get_xyz.detach(), pc.get_scaling.detach(), c, radii,
                                pc.get_is_sky.reshape(-1).contiguous()).cpu().double()
    x = pc.get_xyz.detach().cpu().double()
    sm = pc.get_scaling.detach().cpu().double().min(1).values
    sky = pc.get_is_sky.reshape(-1).cpu()
    cc = c.cpu().double()
    for v in range(V):
        vis = radii[v].cpu() > 0
        fg, sk = vis & ~sky, vis & sky
        depth = x @ cc[v, :3] + cc[v, 3]
        assert sums[v, 0] == int(fg.sum()) and sums[v, 1] == int(sk.sum())
        for k, ref in ((2, sm[fg].sum()), (3, depth[sk].sum()), (4, depth[fg].sum())):
            assert abs(float(sums[v, k] - ref)) <= 1e-5 * max(1.0, float(abs(ref))) + 1e-3, (v, k)
    assert _lib.lib().gsr_view_regularisers_forward(P, 9, None, None, None, None, None, None, None) != 0


@pytest.mark.parametrize("deg", [0, 1, 2, 3, 4])
def test_sh_basis_fused_matches_torch(deg):
    from gsr import train
    d = torch.rand(777, 3, device="cuda") * 2 - 1
    got = train.sh_basis_fused(deg, d)
    ref = train.sh_basis(deg, d / d.norm(dim=-1, keepdim=True))
    assert got.shape == ref.shape
    assert float((got - ref).abs().max()) < 2e-6


def test_sky_xyz_fused_matches_torch():
    """Angles inside and outside the clamp ranges (and exactly on the bounds): positions and
    gradients of the angles and the radius equal the elementwise composition's."""
    from gsr import train
    g = torch.Generator().manual_seed(4)
    N = 20000
    ang = torch.stack([torch.rand(N, generator=g) * 2.4 - 0.4, torch.rand(N, generator=g) * 4.0 - 2.0], 1)
    ang[:5, 0] = torch.tensor([0.0, torch.pi / 2, -0.1, 1.7, 0.3])
    ang[5:10, 1] = torch.tensor([-torch.pi / 2, torch.pi / 2, -1.6, 1.6, 0.0])
    ang = ang.cuda().requires_grad_(True)
    rad = torch.tensor([31.5], device="cuda", requires_grad=True)
    ctr = torch.tensor([0.3, -1.0, 2.0], device="cuda")
    w = torch.randn(N, 3, device="cuda")
    got = train.sky_xyz(ang, rad, ctr, fused=True)
    ga, gr = torch.autograd.grad((got * w).sum(), [ang, rad])
    ref = train.sky_xyz(ang, rad, ctr, fused=False)
    ra, rr = torch.autograd.grad((ref * w).sum(), [ang, rad])
    assert float((got - ref).abs().max()) < 1e-5 * 32
    e = float((ga - ra).abs().max() / ra.abs().max())
    assert e < 1e-5, e
    assert abs(float(gr - rr)) <= 1e-5 * abs(float(rr)) + 1e-3
    assert float(ga[2, 0]) == 0.0 and float(ga[3, 0]) == 0.0 and float(ga[7, 1]) == 0.0 and float(ga[8, 1]) == 0.0


def test_densify_stats_fused_matches_per_view():
    from gsr import dp
    P, V = 30011, 5
    g = torch.Generator().manual_seed(2)
    grads = [torch.randn(P, 3, generator=g).cuda() for _ in range(V)]
    radii = [((torch.rand(P, generator=g) < 0.5) * torch.randint(1, 40, (P,), generator=g)).int().cuda()
             for _ in range(V)]
    a, b = dp.StepStats(P, "cuda"), dp.StepStats(P, "cuda")
    for st in (a, b):
        st.d["xyz_gradient_accum"].uniform_()
        st.d["max_radii2D"].fill_(7.0)
    b.d = {k: v.clone() for k, v in a.d.items()}
    a.add_views(grads, radii)
    for gr, r in zip(grads, radii):
        b.add_view(gr, r)
    torch.cuda.synchronize()
    assert torch.equal(a.d["denom"], b.d["denom"])
    assert torch.equal(a.d["max_radii2D"], b.d["max_radii2D"])
    np.testing.assert_allclose(a.d["xyz_gradient_accum"].cpu().numpy(), b.d["xyz_gradient_accum"].cpu().numpy(),
                               rtol=1e-6, atol=0)


@pytest.mark.parametrize("layout", ["tail", "interleaved", "no_sky"])
def test_fused_activations_match_torch(layout):
    """RelitScene.model_fused (gsr_activations_*) against model()'s PyTorch activations:
    values, and the raw parameters' gradients it writes into the flat gradient against
    autograd's, for the sky rows last, interleaved, and absent; angles past the clamp bounds
    included."""
    from gsr import train
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(17)
    P = 5003
    if layout == "tail":
        is_sky = torch.zeros(P, dtype=torch.bool)
        is_sky[P - 700:] = True
    elif layout == "interleaved":
        is_sky = torch.rand(P, generator=g) < 0.15
    else:
        is_sky = torch.zeros(P, dtype=torch.bool)
    nf = int((~is_sky).sum())
    xyz = torch.randn(P, 3, generator=g) * 2 + torch.tensor([0.0, 0.0, 5.0])
    xyz[is_sky] = torch.nn.functional.normalize(torch.randn(int(is_sky.sum()), 3, generator=g), dim=-1) * 30
    scene = train.RelitScene(xyz, torch.randn(P, 3, generator=g) - 3, torch.randn(P, 4, generator=g),
                             torch.randn(P, 1, generator=g), torch.randn(nf, 3, generator=g), torch.randn(nf, 1, generator=g),
                             torch.randn(nf, 1, generator=g), is_sky, 2, dev)
    if int(is_sky.sum()):
        with torch.no_grad():
            a = scene.fp.params["sky_angles"]
            a[:7, 0] = torch.tensor([-0.2, 0.0, torch.pi / 2, 1.7, 0.4, 0.4, 0.4])
            a[:7, 1] = torch.tensor([0.1, 0.1, 0.1, 0.1, -1.8, torch.pi / 2, 1.9])
    names = ["get_xyz", "get_scaling", "get_rotation", "get_opacity", "get_albedo", "get_roughness", "get_metalness"]
    ref = scene.model()
    got = scene.model_fused()
    for n in names:
        a, b = getattr(got, n), getattr(ref, n)
        assert a.shape == b.shape, n
        assert float((a - b).abs().max()) <= 2e-6 * max(1.0, float(b.abs().max())), n
    ws = [torch.randn(getattr(ref, n).shape, generator=g).to(dev) for n in names]
    scene.fp.zero_grad()
    sum((getattr(got, n) * w).sum() for n, w in zip(names, ws)).backward()
    fused = scene.fp.grad.clone()
    scene.fp.check_grads_in_place()
    scene.fp.zero_grad()
    sum((getattr(ref, n) * w).sum() for n, w in zip(names, ws)).backward()
    torch.cuda.synchronize()
    for name in ("xyz", "sky_angles", "sky_radius", "scaling", "rotation", "opacity", "albedo", "roughness",
                 "metalness"):
        i = scene.fp.names.index(name)
        a = fused[scene.fp.offsets[i]:scene.fp.ends[i]].cpu()
        b = scene.fp.grad[scene.fp.offsets[i]:scene.fp.ends[i]].cpu()
        if b.numel() == 0:  # an empty group (no sky rows)
            assert a.numel() == 0, name
            continue
        if float(b.abs().max()) == 0:
            assert float(a.abs().max()) == 0, name
            continue
        e = float((a - b).norm() / b.norm())
        assert e < 1e-5, (name, e)


@pytest.mark.parametrize("sums", [True, False])
def test_dp_add_views_fused_matches_torch(sums):
    """gsr.dp.add_views (train_step's statistics, gsr_densify_stats in launches of up to 8
    views) against its PyTorch path over 11 views; sums=False: max radii alone (past
    densify_until_iter, train.py:130 vs :143-144) -- accum and denom untouched."""
    from gsr import dp
    P, V = 20011, 11
    g = torch.Generator().manual_seed(4)
    grads = [torch.randn(P, 3, generator=g) for _ in range(V)]
    radii = [((torch.rand(P, generator=g) < 0.5) * torch.randint(1, 40, (P,), generator=g)).int() for _ in range(V)]
    base = {"a": torch.rand(P, 1, generator=g), "d": torch.randint(0, 5, (P, 1), generator=g).float(),
            "m": torch.full((P,), 7.0)}
    cpu = {k: v.clone() for k, v in base.items()}
    gpu = {k: v.cuda() for k, v in base.items()}
    dp.add_views(cpu["a"] if sums else None, cpu["d"] if sums else None, cpu["m"], grads, radii)
    dp.add_views(gpu["a"] if sums else None, gpu["d"] if sums else None, gpu["m"], [t.cuda() for t in grads],
                 [r.cuda() for r in radii])
    torch.cuda.synchronize()
    assert torch.equal(gpu["m"].cpu(), cpu["m"])
    assert torch.equal(gpu["d"].cpu(), cpu["d"])
    np.testing.assert_allclose(gpu["a"].cpu().numpy(), cpu["a"].numpy(), rtol=1e-6, atol=0)
    if not sums:
        assert torch.equal(gpu["a"].cpu(), base["a"]) and torch.equal(gpu["d"].cpu(), base["d"])
