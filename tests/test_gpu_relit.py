"""Fused relit features (relit_shade.relit_features) and the fused render()
(gsr.relit.render).

* Geometry columns (depth, flipped minimum-scale normal) against the goldens the
  reference's own code produced (tests/golden/geometry.npz: GaussianModel.get_depth,
  get_minimum_axis + flip_align_view).
* The whole feature row and its gradients against a PyTorch composition of render()'s
  steps (gaussian_renderer/__init__.py:120-200) around the drop-in shade op
  (relit_shade.shade, itself pinned by tests/golden/shade.npz).
* gsr.relit.render against render()'s own call sequence on the drop-in rasterizer
  (six separate calls): every output image and every gradient.
"""
import math
import os
import types

import numpy as np
import pytest
import torch

from helpers import make_case

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
C0, C1 = 0.28209479177387814, 0.4886025119029199


def _rel(a, b):
    a, b = a.detach(), b.detach()
    return float(torch.linalg.norm((a - b).double()) / torch.linalg.norm(b.double()).clamp_min(1e-30))


def _light(deg=4, seed=0):
    import relit_shade
    g = torch.Generator().manual_seed(seed)
    base = torch.randn((deg + 1) ** 2, 3, generator=g) * 0.3
    base[0] = 1.0
    return relit_shade.EnvironmentLight(base.cuda(), sh_degree=deg)


@pytest.mark.parametrize("cam", [0, 1, 2])
def test_geometry_columns_match_reference_goldens(cam):
    import relit_shade
    d = np.load(os.path.join(GOLD, "geometry.npz"), allow_pickle=False)
    t = lambda k: torch.from_numpy(np.ascontiguousarray(d[k])).float().cuda()
    P = d["xyz"].shape[0]
    feat = relit_shade.relit_features(t("xyz"), t("rotations"), t("scales"), torch.ones(P, dtype=torch.bool).cuda(),
                                      torch.zeros(0, 3).cuda(), torch.zeros(0, 1).cuda(), torch.zeros(0, 1).cuda(),
                                      _light(), t(f"cam{cam}/campos"), t(f"cam{cam}/viewmatrix"), fix_sky=True)
    np.testing.assert_allclose(feat[:, 9].cpu().numpy(), d[f"cam{cam}/depth"].reshape(-1), rtol=2e-6, atol=2e-6)
    np.testing.assert_allclose(feat[:, 10:13].cpu().numpy(), 0.5 * d[f"cam{cam}/normal_flipped"] + 0.5, rtol=0,
                               atol=1e-6)
    assert torch.equal(feat[:, 0:3], torch.ones(P, 3).cuda()) and torch.equal(feat[:, 13], torch.ones(P).cuda())
    assert not feat[:, 3:9].any() and not feat[:, 14:].any()


def _scene(P=4000, n_sky=400, seed=0):
    g = torch.Generator().manual_seed(seed)
    xyz = torch.randn(P, 3, generator=g) * 1.5 + torch.tensor([0.0, 0.0, 5.0])
    q = torch.nn.functional.normalize(torch.randn(P, 4, generator=g), dim=1)
    s = torch.exp(torch.randn(P, 3, generator=g) * 0.5 - 3.0)
    is_sky = torch.zeros(P, dtype=torch.bool)
    is_sky[torch.randperm(P, generator=g)[:n_sky]] = True
    N = P - n_sky
    mat = dict(albedo=torch.rand(N, 3, generator=g), roughness=torch.rand(N, 1, generator=g) * 0.9 + 0.05,
               metalness=torch.rand(N, 1, generator=g))
    sky_sh = torch.randn(1, 4, 3, generator=g) * 0.4
    cam, _ = make_case(P=10, W=64, H=48, camera="orbit")
    c = lambda x: x.cuda()
    return (c(xyz), c(q), c(s), c(is_sky), {k: c(v) for k, v in mat.items()}, c(sky_sh),
            cam.camera_center.cuda(), cam.world_view_transform.cuda())


def _composition(xyz, q, s, is_sky, mat, sky_sh, light, campos, wvt, specular=True, fix_sky=False):
    """render()'s per-Gaussian steps in PyTorch (gaussian_renderer/__init__.py:120-200) with
    the drop-in shade."""
    import relit_shade
    d = xyz - campos[None]
    dirn = d / torch.sqrt(torch.clamp((d * d).sum(-1, keepdim=True), min=1e-20))
    qn = q / torch.sqrt((q * q).sum(1, keepdim=True))
    r, x, y, z = qn.unbind(1)
    R = torch.stack([torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], -1),
                     torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], -1),
                     torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1)], 1)
    idx = s.min(dim=-1)[1][..., None, None].expand(-1, 3, -1)
    axis = R.gather(2, idx).squeeze(2)
    keep = (axis * -dirn).sum(-1, keepdim=True) >= 0
    n = axis * torch.where(keep, 1, -1)
    fg = ~is_sky
    P = xyz.shape[0]
    cols = torch.zeros(P, 3, device="cuda")
    dif = torch.zeros(P, 3, device="cuda")
    spe = torch.zeros(P, 3, device="cuda")
    if fg.any():  # render() shades only when it has foreground Gaussians
        rgb, ex = relit_shade.shade(light, xyz[fg][None, None], n[fg][None, None], mat["albedo"][None, None],
                                    campos.expand(int(fg.sum()), 3)[None, None], mat["roughness"][None, None],
                                    mat["metalness"][None, None], specular=specular)
        cols[fg] = rgb[0, 0]
        dif[fg] = ex["diffuse"][0, 0]
        spe[fg] = ex["specular"][0, 0]
    if fix_sky:
        cols[is_sky] = 1.0
    else:
        dd = dirn[is_sky]
        sh = sky_sh[0]
        v = C0 * sh[0] - C1 * dd[:, 1:2] * sh[1] + C1 * dd[:, 2:3] * sh[2] - C1 * dd[:, 0:1] * sh[3]
        cols[is_sky] = torch.clamp_min(v + 0.5, 0.0)
    p_hom = torch.cat([xyz, torch.ones_like(xyz[:, :1])], -1).unsqueeze(-1)
    depth = torch.matmul(wvt.transpose(0, 1), p_hom)[:, 2]
    return torch.cat([cols, dif, spe, depth, 0.5 * n + 0.5, torch.ones(P, 1, device="cuda")], 1)


@pytest.mark.parametrize("specular,fix_sky,P,n_sky", [(True, False, 4000, 400), (False, False, 4000, 400),
                                                      (True, True, 4000, 400),
                                                      # edge cases of the fused kernels' fg/sky ranks: no sky,
                                                      # a ragged last workgroup, a lone foreground Gaussian,
                                                      # no foreground at all
                                                      (True, False, 4000, 0), (True, False, 257, 1),
                                                      (True, False, 300, 299), (True, False, 300, 300)])
def test_relit_features_match_composition(specular, fix_sky, P, n_sky):
    import relit_shade
    xyz, q, s, is_sky, mat, sky_sh, campos, wvt = _scene(P=P, n_sky=n_sky)
    light = _light()
    leaves = lambda: [t.clone().requires_grad_(True) for t in (xyz, q, mat["albedo"], mat["roughness"],
                                                                 mat["metalness"], light.base, sky_sh)]
    g = torch.Generator(device="cuda").manual_seed(5)
    w = torch.randn(xyz.shape[0], 14, device="cuda", generator=g)

    def run(fn):
        x, qq, al, kr, km, base, ssh = leaves()
        lt = relit_shade.EnvironmentLight(base, sh_degree=4)
        m = dict(albedo=al, roughness=kr, metalness=km)
        f = fn(x, qq, m, lt, ssh)[:, :14]
        (f * w).sum().backward()
        return f.detach(), [x.grad, qq.grad, al.grad, kr.grad, km.grad, base.grad, ssh.grad]

    f_fused, g_fused = run(lambda x, qq, m, lt, ssh: relit_shade.relit_features(
        x, qq, s, is_sky, m["albedo"], m["roughness"], m["metalness"], lt, campos, wvt, ssh, 1, specular, fix_sky))
    f_ref, g_ref = run(lambda x, qq, m, lt, ssh: _composition(x, qq, s, is_sky, m, ssh, lt, campos, wvt, specular,
                                                               fix_sky))
    assert _rel(f_fused, f_ref) < 1e-6
    names = ["xyz", "rotation", "albedo", "roughness", "metalness", "base", "sky_sh"]
    for name, a, b in zip(names, g_fused, g_ref):
        if b is None or not b.any():
            assert a is None or not a.any(), name
            continue
        assert _rel(a, b) < 2e-5, (name, _rel(a, b))


class _Model:
    """The GaussianModel properties render() reads."""

    def __init__(self, xyz, q, s, is_sky, mat, opacity):
        self.get_xyz, self.get_rotation, self.get_scaling, self.get_opacity = xyz, q, s, opacity
        self.get_is_sky = is_sky[:, None]
        self.get_albedo, self.get_roughness, self.get_metalness = mat["albedo"], mat["roughness"], mat["metalness"]


def _reference_render(view, pc, light, sky_sh, bg, debug):
    """render()'s call sequence (gaussian_renderer/__init__.py:69-280) on the drop-in
    rasterizer, one call per image."""
    import diff_gaussian_rasterization as dgr
    from gsr.relit import depth_to_normal
    sp = torch.zeros_like(pc.get_xyz, requires_grad=True) + 0
    sp.retain_grad()
    st = dgr.GaussianRasterizationSettings(
        image_height=view.image_height, image_width=view.image_width, tanfovx=math.tan(view.FoVx * 0.5),
        tanfovy=math.tan(view.FoVy * 0.5), bg=bg, scale_modifier=1.0, viewmatrix=view.world_view_transform,
        projmatrix=view.full_proj_transform, sh_degree=-1, campos=view.camera_center, prefiltered=False)
    rast = dgr.GaussianRasterizer(st)
    is_sky = pc.get_is_sky.squeeze()
    f = _composition(pc.get_xyz, pc.get_rotation, pc.get_scaling, is_sky,
                     dict(albedo=pc.get_albedo, roughness=pc.get_roughness, metalness=pc.get_metalness), sky_sh,
                     light, view.camera_center, view.world_view_transform)
    call = lambda col, r=rast: r(means3D=pc.get_xyz, means2D=sp, shs=None, colors_precomp=col.contiguous(),
                                 opacities=pc.get_opacity, scales=pc.get_scaling, rotations=pc.get_rotation)
    img, radii = call(f[:, 0:3])
    out = {"render": img, "viewspace_points": sp, "visibility_filter": radii > 0, "radii": radii}
    ex = {"diffuse_color": f[:, 3:6], "specular_color": f[:, 6:9], "depth": f[:, 9:10].repeat(1, 3),
          "normal": f[:, 10:13]}
    if debug:
        P = pc.get_xyz.shape[0]
        fg = ~is_sky
        r_all = torch.zeros((P, 1), device="cuda")
        r_all[fg] = pc.get_roughness
        m_all = torch.zeros((P, 1), device="cuda")
        m_all[fg] = pc.get_metalness
        a_all = torch.ones_like(pc.get_xyz)
        a_all[fg] = pc.get_albedo
        ex.update({"sky_color": f[:, 0:3] * is_sky[:, None].float(), "roughness": r_all.repeat(1, 3),
                   "metalness": m_all.repeat(1, 3), "albedo": a_all})
    sky_mask = view.sky_mask.cuda().squeeze()
    for k, v in ex.items():
        im = call(v)[0]
        if k == "normal":
            im = (im - 0.5) * 2.
            im = im * sky_mask + torch.ones_like(im) * (1 - sky_mask)
        out[k] = im
    ra = dgr.GaussianRasterizer(st._replace(bg=torch.zeros(3, device="cuda")))
    out["alpha"] = call(torch.ones_like(pc.get_xyz), ra)[0]
    nr = depth_to_normal(view, (out["depth"][0] * sky_mask).unsqueeze(0)).permute(2, 0, 1)
    nr = nr * out["alpha"].detach()
    out["normal_ref"] = nr + torch.ones_like(nr) * (1 - sky_mask)
    return out


@pytest.mark.parametrize("bg,debug,n_sky", [((0.0, 0.0, 0.0), False, 600), ((1.0, 1.0, 1.0), True, 600),
                                            ((0.2, 0.5, 0.9), False, 600), ((0.2, 0.5, 0.9), True, 600),
                                            # a scene without sky, and one of sky alone
                                            ((0.2, 0.5, 0.9), True, 0), ((0.0, 0.0, 0.0), True, 6000)])
def test_fused_render_matches_reference_calls(bg, debug, n_sky):
    from gsr import relit
    xyz, q, s, is_sky, mat, sky_sh, _, _ = _scene(P=6000, n_sky=n_sky, seed=3)
    cam, _ = make_case(P=10, W=160, H=120, camera="orbit")
    g = torch.Generator().manual_seed(8)
    sky_mask = (torch.rand(1, 120, 160, generator=g) > 0.2).float()
    view = types.SimpleNamespace(image_width=160, image_height=120, FoVx=cam.FoVx, FoVy=cam.FoVy,
                                 world_view_transform=cam.world_view_transform.cuda(),
                                 full_proj_transform=cam.full_proj_transform.cuda(),
                                 camera_center=cam.camera_center.cuda(), sky_mask=sky_mask)
    opacity = torch.rand(xyz.shape[0], 1, generator=g).cuda() * 0.9 + 0.05
    light = _light()
    pipe = types.SimpleNamespace(compute_cov3D_python=False)
    bgt = torch.tensor(bg, device="cuda")
    wts = {}

    def run(fn):
        leaves = [t.clone().requires_grad_(True) for t in (xyz, q, mat["albedo"], light.base, opacity)]
        pc = _Model(leaves[0], leaves[1], s, is_sky, dict(mat, albedo=leaves[2]), leaves[4])
        import relit_shade
        lt = relit_shade.EnvironmentLight(leaves[3], sh_degree=4)
        out = fn(pc, lt)
        loss = 0.0
        gen = torch.Generator(device="cuda").manual_seed(4)
        for k in sorted(out):
            if k in ("viewspace_points", "visibility_filter", "radii"):
                continue
            wts.setdefault(k, torch.randn(out[k].shape, device="cuda", generator=gen))
            loss = loss + (out[k] * wts[k]).sum()
        loss.backward()
        return out, [t.grad for t in leaves] + [out["viewspace_points"].grad]

    o_f, g_f = run(lambda pc, lt: relit.render(view, pc, lt, sky_sh, 1, pipe, bgt, debug=debug))
    o_r, g_r = run(lambda pc, lt: _reference_render(view, pc, lt, sky_sh, bgt, debug))
    assert sorted(o_f) == sorted(o_r)
    assert torch.equal(o_f["radii"], o_r["radii"])
    for k in o_r:
        if k in ("viewspace_points", "visibility_filter", "radii"):
            continue
        assert o_f[k].shape == o_r[k].shape, k
        assert _rel(o_f[k], o_r[k]) < 1e-5, (k, _rel(o_f[k], o_r[k]))
    for name, a, b in zip(["xyz", "rotation", "albedo", "base", "opacity", "means2D"], g_f, g_r):
        if b is None or not b.any():  # no foreground: nothing reaches albedo or the light
            assert a is None or not a.any(), name
            continue
        assert _rel(a, b) < 1e-4, (name, _rel(a, b))


@pytest.mark.parametrize("normal_view", [False, True])
def test_epilogue_matches_torch_restatement(normal_view):
    """gsr_relit_epilogue (normal remap + sky mask + normal_ref) against render()'s PyTorch
    tail (gaussian_renderer/__init__.py:226-276 with depth_to_normal), forward and backward."""
    from gsr import relit
    from gsr import scenes
    H, W = 70, 96
    R, T = scenes.look_at_rotation([0.4, -0.3, -1.0], [0.0, 0.0, 5.0])
    cam = scenes.make_camera(W, H, 1.1, 0.85, R=R, T=T)
    view = types.SimpleNamespace(world_view_transform=cam.world_view_transform.cuda(), image_width=W, image_height=H,
                                 FoVx=cam.FoVx, FoVy=cam.FoVy)
    g = torch.Generator().manual_seed(3)
    n01 = torch.rand(3, H, W, generator=g).cuda()
    depth = (torch.rand(H, W, generator=g) * 0.5 + 4.0).cuda()
    alpha = torch.rand(H, W, generator=g).cuda()
    sky = (torch.rand(H, W, generator=g) > 0.15).float().cuda()
    w1, w2 = torch.randn(3, H, W, generator=g).cuda(), torch.randn(3, H, W, generator=g).cuda()

    def torch_tail(n, d):
        nrm = (n - 0.5) * 2.
        if normal_view:
            nrm = -nrm.clone()
        nrm = nrm * sky + torch.ones_like(nrm) * (1 - sky)
        nr = relit.depth_to_normal(view, (d * sky).unsqueeze(0)).permute(2, 0, 1) * alpha
        return nrm, nr + torch.ones_like(nr) * (1 - sky)

    def run(fn):
        n, d = n01.clone().requires_grad_(True), depth.clone().requires_grad_(True)
        a, b = fn(n, d)
        ((a * w1).sum() + (b * w2).sum()).backward()
        return a.detach(), b.detach(), n.grad, d.grad

    got = run(lambda n, d: relit._Epilogue.apply(n, d, alpha, sky, relit._epilogue_camera(view), normal_view))
    want = run(torch_tail)
    for name, a, b in zip(("normal", "normal_ref", "d_n01", "d_depth"), got, want):
        assert _rel(a, b) < 1e-5, (name, _rel(a, b))
