"""The relightable render() step on the fused path (SURVEY §8f #1 + #2).

`render` has the signature and outputs of the reference's gaussian_renderer.render
(gaussian_renderer/__init__.py:69-280), and computes them with three ops instead of a
chain of ~60 PyTorch kernels and 6-10 rasterizer calls:

  1. relit_shade.relit_features -- every per-Gaussian channel render() prepares (shaded
     colour, diffuse, specular, depth, normal, alpha; sky colours for sky Gaussians) as
     [P, 16] rows, one HIP pass each way;
  2. diff_gaussian_rasterization.rasterize_channels -- one geometry pass and one
     multi-channel composite of all images (the debug extras add a second 16-channel group);
  3. the reference's image-space post-processing (normal remap, sky masking, normal_ref
     from the depth image), restated in PyTorch.

Each image equals what the reference's separate call produces from the same per-Gaussian
colours (tests/test_gpu_relit.py).  Opt-in: callers import this `render` in place of
gaussian_renderer.render.
"""
import math

import torch


def depths_to_points(view, depthmap):
    """graphics_utils.py:141-156: back-project a depth map through the camera.  The
    reference's `pixels @ K^-1^T @ R^T` is written as three broadcast multiply-adds per
    pixel (two [H*W,3] @ [3,3] GEMMs cost ~130 us each on hipBLASLt at 1080p)."""
    c2w = view.world_view_transform.T.inverse()
    W, H = view.image_width, view.image_height
    fx = W / (2 * math.tan(view.FoVx / 2.))
    fy = H / (2 * math.tan(view.FoVy / 2.))
    dev = depthmap.device
    intrins = torch.tensor([[fx, 0., W / 2.], [0., fy, H / 2.], [0., 0., 1.0]], device=dev).float()
    M = intrins.inverse().T @ c2w[:3, :3].T  # [3, 3]: rays_d = [x, y, 1] @ M
    gx = torch.arange(W, device=dev).float()
    gy = torch.arange(H, device=dev).float()
    rays_d = (gx[None, :, None] * M[0] + gy[:, None, None] * M[1] + M[2]).reshape(-1, 3)
    return depthmap.reshape(-1, 1) * rays_d + c2w[:3, 3]


def depth_to_normal(view, depth):
    """graphics_utils.py:158-169: normals from the depth image by central differences."""
    points = depths_to_points(view, depth).reshape(*depth.shape[1:], 3)
    out = torch.zeros_like(points)
    dx = points[2:, 1:-1] - points[:-2, 1:-1]
    dy = points[1:-1, 2:] - points[1:-1, :-2]
    out[1:-1, 1:-1, :] = torch.nn.functional.normalize(torch.cross(dx, dy, dim=-1), dim=-1)
    return out


def _epilogue_camera(view):
    """cam12 for gsr_relit_epilogue: rows of K^-1^T R^T (rays = x M0 + y M1 + M2) and the
    camera centre, as depths_to_points builds them.  Cached on the view object (keyed on the
    matrix object and its version), so a training loop pays its host round trip once."""
    wvt = view.world_view_transform
    key = (wvt._version, view.image_width, view.image_height, view.FoVx, view.FoVy)
    hit = getattr(view, "_gsr_cam12", None)
    if hit is not None and hit[0] is wvt and hit[1] == key:
        return hit[2]
    cam12 = _epilogue_camera_uncached(view)
    try:
        view._gsr_cam12 = (wvt, key, cam12)
    except AttributeError:
        pass
    return cam12


def _epilogue_camera_uncached(view):
    c2w = view.world_view_transform.T.inverse().double()
    W, H = view.image_width, view.image_height
    fx = W / (2 * math.tan(view.FoVx / 2.))
    fy = H / (2 * math.tan(view.FoVy / 2.))
    K = torch.tensor([[fx, 0., W / 2.], [0., fy, H / 2.], [0., 0., 1.0]], dtype=torch.float64, device=c2w.device)
    M = K.inverse().T @ c2w[:3, :3].T
    return torch.cat([M.reshape(-1), c2w[:3, 3]]).float().cpu().contiguous()


class _Epilogue(torch.autograd.Function):
    """render()'s image-space tail on the GPU (gsr_relit_epilogue): (n01 [3,H,W], depth
    [H,W], alpha [H,W] (detached), sky [H,W]) -> (normal, normal_ref), both [3,H,W]."""

    @staticmethod
    def forward(ctx, n01, depth, alpha, sky, cam12, normal_view, dest=None):
        from . import _lib
        H, W = depth.shape
        n01, depth, alpha, sky = (t.float().contiguous() for t in (n01, depth, alpha, sky))
        normal = torch.empty((3, H, W), dtype=torch.float32, device=depth.device)
        nref = torch.empty_like(normal)
        _lib.check(_lib.lib().gsr_relit_epilogue(W, H, cam12.data_ptr(), n01.data_ptr(), depth.data_ptr(),
                                                 alpha.data_ptr(), sky.data_ptr(), int(normal_view),
                                                 normal.data_ptr(), nref.data_ptr(), _lib.stream_of(depth.device)),
                   "gsr_relit_epilogue")
        ctx.save_for_backward(depth, alpha, sky, cam12)
        ctx.normal_view = normal_view
        ctx.dest = dest  # (n01's, depth's) composite groups: their gradients go to its GradSlab
        return normal, nref

    @staticmethod
    def backward(ctx, g_normal, g_nref):
        from . import _lib
        depth, alpha, sky, cam12 = ctx.saved_tensors
        H, W = depth.shape
        c = lambda t: None if t is None else t.float().contiguous()
        g_normal, g_nref = c(g_normal), c(g_nref)
        d_n01 = d_depth = None
        if ctx.needs_input_grad[0]:
            d_n01 = slab_take(ctx.dest[0]) if ctx.dest else None
            if d_n01 is None or d_n01.shape != (3, H, W):
                d_n01 = torch.empty((3, H, W), dtype=torch.float32, device=depth.device)
        if ctx.needs_input_grad[1]:
            d_depth = slab_take(ctx.dest[1]) if ctx.dest else None
            d_depth = torch.empty_like(depth) if d_depth is None or d_depth.numel() != H * W else d_depth.view(H, W)
        ptr = lambda t: None if t is None else t.data_ptr()
        if d_n01 is not None or d_depth is not None:
            _lib.check(_lib.lib().gsr_relit_epilogue_backward(
                W, H, cam12.data_ptr(), depth.data_ptr(), alpha.data_ptr(), sky.data_ptr(), int(ctx.normal_view),
                ptr(g_normal), ptr(g_nref), ptr(d_n01), ptr(d_depth), _lib.stream_of(depth.device)),
                "gsr_relit_epilogue_backward")
        return d_n01, d_depth, None, None, None, None, None


_GREY = {}
_ZEROS = {}
_BGCAT = {}


def _zero_rows(like, dev=None, n=None):
    """Zeros shaped like ``like`` [P, 3] (an expanded view of one cached zero: no fill kernel
    per view), or a cached zero vector of n elements."""
    dev = like.device if like is not None else dev
    z = _ZEROS.get(str(dev))
    if z is None:
        z = _ZEROS[str(dev)] = torch.zeros(16, dtype=torch.float32, device=dev)
        if z.is_cuda:  # complete before another stream reads it
            torch.cuda.current_stream(z.device).synchronize()
    if like is None:
        return z[:n]
    return z[:1].view(1, 1).expand(like.shape[0], like.shape[1])


def _bg_cat(bg_color, widths, parts):
    """torch.cat(parts): the composite's background vector, a function of the background
    tensor (identity and version) and the channel widths; cached, since a training run
    renders every view over the same background."""
    key = (id(bg_color), bg_color._version, tuple(widths), str(bg_color.device))
    hit = _BGCAT.get(key)
    if hit is not None and hit[0] is bg_color:
        return hit[1]
    out = torch.cat(parts)
    if out.is_cuda:  # complete before another view's stream reads it
        torch.cuda.current_stream(out.device).synchronize()
    if len(_BGCAT) > 16:
        _BGCAT.clear()
    _BGCAT[key] = (bg_color, out)
    return out


def _is_grey(bg_color):
    """Whether every background channel is equal (one composite channel then serves a value
    render() repeats over three).  Cached on the tensor's identity and version: the check
    reads the device tensor, i.e. it is a host synchronisation, and the background of a
    training run never changes."""
    hit = _GREY.get(id(bg_color))
    if hit is not None and hit[0] is bg_color and hit[1] == bg_color._version:
        return hit[2]
    bg = bg_color.reshape(-1).float()
    grey = bool((bg == bg[0]).all())
    if len(_GREY) > 16:
        _GREY.clear()
    _GREY[id(bg_color)] = (bg_color, bg_color._version, grey)
    return grey


class GradSlab:
    """The gradient image of one composite [C,H,W], handed out in channel groups: a consumer
    of a group (the fused view objective, the epilogue) writes its gradient straight into
    the group's rows instead of a tensor of its own that the split's backward would then
    copy.  Each group is handed out once (a second consumer, or a second backward over the
    same graph, gets None and allocates as usual; the split then copies)."""

    def __init__(self, shape, device):
        self.shape, self.device = tuple(shape), device
        self.t = None
        self.taken = set()

    def take(self, c0: int, k: int):
        if c0 in self.taken:
            return None
        self.taken.add(c0)
        if self.t is None:
            self.t = torch.empty(self.shape, dtype=torch.float32, device=self.device)
        return self.t[c0:c0 + k]

    def holds(self, g, c0: int) -> bool:
        return (self.t is not None and c0 in self.taken and g.dtype == torch.float32 and g.is_contiguous()
                and g.data_ptr() == self.t[c0].data_ptr())


def slab_take(t, k=None):
    """The GradSlab rows reserved for tensor ``t`` (a group of a composite split by render()),
    or None."""
    tag = getattr(t, "_gsr_slab", None)
    if tag is None:
        return None
    slab, c0, kk = tag
    return slab.take(c0, kk if k is None else k)


class _SplitChannels(torch.autograd.Function):
    """The composite image [C,H,W] split into consecutive channel groups (views).  The
    backward returns the GradSlab its consumers wrote into when every group's gradient is
    its slab rows (zeroing the groups with none); otherwise it writes each group's gradient
    into one [C,H,W] tensor (zeros only where a group has none) instead of autograd's
    full-size zero tensor + add per slice."""

    @staticmethod
    def forward(ctx, image, widths, slab):
        ctx.set_materialize_grads(False)  # groups without a gradient arrive as None, not zeros
        ctx.widths = widths
        ctx.shape = image.shape
        ctx.slab = slab
        out, c = [], 0
        for k in widths:
            out.append(image[c:c + k])
            c += k
        return tuple(out)

    @staticmethod
    def backward(ctx, *grads):
        slab, offs, c = ctx.slab, [], 0
        for k in ctx.widths:
            offs.append(c)
            c += k
        if slab is not None and slab.t is not None and all(t is None or slab.holds(t, c0)
                                                           for t, c0 in zip(grads, offs)):
            g = slab.t
            for k, t, c0 in zip(ctx.widths, grads, offs):
                if t is None:
                    g[c0:c0 + k].zero_()
            if c < g.shape[0]:
                g[c:].zero_()
            return g, None, None
        g = torch.empty(ctx.shape, dtype=torch.float32, device=next(t for t in grads if t is not None).device) \
            if any(t is not None for t in grads) else None
        if g is None:
            return None, None, None
        for k, t, c0 in zip(ctx.widths, grads, offs):
            if t is None:
                g[c0:c0 + k].zero_()
            else:
                g[c0:c0 + k].copy_(t)
        if c < g.shape[0]:
            g[c:].zero_()
        return g, None, None


def render(viewpoint_camera, pc, envlight, sky_sh, sky_sh_degree, pipe, bg_color, scaling_modifier=1.0, debug=True,
           specular=True, fix_sky=False, normal_view=False):
    """gaussian_renderer/__init__.py:69-280 on the fused path (same arguments, same output
    dictionary: render, viewspace_points, visibility_filter, radii, diffuse_color,
    specular_color, depth, normal, alpha, normal_ref and, with debug, sky_color, roughness,
    metalness, albedo)."""
    import diff_gaussian_rasterization as dgr
    import relit_shade

    # a leaf (the reference adds 0 to make it a non-leaf and retains its gradient: the same
    # .grad after backward, without a full-size add kernel per view)
    # (its values are never read, only its gradient: an expanded zero, no fill kernel)
    screenspace_points = _zero_rows(pc.get_xyz).requires_grad_(True)
    tanfovx = math.tan(viewpoint_camera.FoVx * 0.5)
    tanfovy = math.tan(viewpoint_camera.FoVy * 0.5)
    settings = dgr.GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=tanfovx, tanfovy=tanfovy, bg=bg_color, scale_modifier=scaling_modifier,
        viewmatrix=viewpoint_camera.world_view_transform, projmatrix=viewpoint_camera.full_proj_transform,
        sh_degree=-1, campos=viewpoint_camera.camera_center, prefiltered=False)

    means3D = pc.get_xyz
    opacity = pc.get_opacity
    empty = torch.Tensor([])
    scales = rotations = cov3D_precomp = empty
    if pipe.compute_cov3D_python:
        cov3D_precomp = pc.get_covariance(scaling_modifier)
    else:
        scales = pc.get_scaling
        rotations = pc.get_rotation
    dev = means3D.device
    sky_mask = viewpoint_camera.sky_mask.to(dev).squeeze()
    is_sky = pc.get_is_sky.squeeze()

    feat = relit_shade.relit_features(means3D, pc.get_rotation, pc.get_scaling, is_sky, pc.get_albedo,
                                      pc.get_roughness, pc.get_metalness, envlight, viewpoint_camera.camera_center,
                                      viewpoint_camera.world_view_transform, sky_sh, sky_sh_degree, specular, fix_sky)
    bg = bg_color.reshape(-1).float()
    # A value repeated over three channels (depth, alpha, roughness, metalness) is one
    # composite channel when the background is grey; otherwise three.
    grey = _is_grey(bg_color)
    zero3 = _zero_rows(None, dev, 3)
    # (name, columns [P, k], background [k]); alpha is rendered with a black background
    chans = [("render", feat[:, 0:3], bg), ("diffuse_color", feat[:, 3:6], bg), ("specular_color", feat[:, 6:9], bg),
             ("depth", feat[:, 9:10], bg), ("normal", feat[:, 10:13], bg), ("alpha", feat[:, 13:14], zero3)]
    if debug:
        P = means3D.shape[0]
        fg = ~is_sky
        rough = torch.zeros((P, 1), device=dev)
        rough[fg] = pc.get_roughness
        metal = torch.zeros((P, 1), device=dev)
        metal[fg] = pc.get_metalness
        alb = torch.ones_like(means3D)
        alb[fg] = pc.get_albedo
        chans += [("sky_color", feat[:, 0:3] * is_sky[:, None].float(), bg), ("roughness", rough, bg),
                  ("metalness", metal, bg), ("albedo", alb, bg)]
    cols, bgs, widths = [], [], []
    for name, cval, b in chans:
        k = cval.shape[1]
        if k == 1 and not (grey or name == "alpha"):
            cval, k = cval.expand(-1, 3), 3
        cols.append(cval)
        bgs.append(b[:k])
        widths.append(k)
    nch = sum(widths)
    # without extras and with a grey background the relit rows are the features as they are
    features = feat if (not debug and grey) else torch.cat(cols, 1)
    image, radii = dgr.rasterize_channels(means3D, screenspace_points, features, opacity, scales, rotations,
                                          cov3D_precomp, _bg_cat(bg_color, widths, bgs), settings, nch=nch)
    H, W = settings.image_height, settings.image_width
    slab = GradSlab(image.shape, image.device)
    parts = _SplitChannels.apply(image, tuple(widths), slab)
    c0 = 0
    for v, k in zip(parts, widths):  # where each group's gradient goes (slab_take)
        v._gsr_slab = (slab, c0, k)
        c0 += k
    imgs = {name: (v.expand(3, H, W) if k == 1 else v) for (name, _, _), k, v in zip(chans, widths, parts)}
    # the depth plane the epilogue reads: a view of a one-channel part (no select of the
    # expanded image, whose backward is a full-size zero tensor + copy + sum)
    planes = {name: (v.view(H, W) if k == 1 else v[0]) for (name, _, _), k, v in zip(chans, widths, parts)}
    out = {"render": imgs["render"], "viewspace_points": screenspace_points, "visibility_filter": radii > 0,
           "radii": radii}
    extras = {k: v for k, v in imgs.items() if k != "render"}
    # normal remap + sky mask and normal_ref from the depth image in one kernel each way
    grp = {name: v for (name, _, _), v in zip(chans, parts)}
    extras["normal"], extras["normal_ref"] = _Epilogue.apply(
        extras["normal"], planes["depth"], planes["alpha"].detach(), sky_mask.float(),
        _epilogue_camera(viewpoint_camera), bool(normal_view), (grp["normal"], grp["depth"]))
    out.update(extras)
    return out


_C0, _C1 = 0.28209479177387814, 0.4886025119029199
_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
       1.445305721320277, -0.5900435899266435)


def eval_sh(deg, sh, dirs):
    """Real SH of degree <= 3 at unit directions (utils/sh_utils.py:81-125, same polynomial
    order): sh [..., C, K], dirs [..., 3] -> [..., C]."""
    assert 0 <= deg <= 3
    res = _C0 * sh[..., 0]
    if deg > 0:
        x, y, z = dirs[..., 0:1], dirs[..., 1:2], dirs[..., 2:3]
        res = res - _C1 * y * sh[..., 1] + _C1 * z * sh[..., 2] - _C1 * x * sh[..., 3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            res = (res + _C2[0] * xy * sh[..., 4] + _C2[1] * yz * sh[..., 5] +
                   _C2[2] * (2.0 * zz - xx - yy) * sh[..., 6] + _C2[3] * xz * sh[..., 7] +
                   _C2[4] * (xx - yy) * sh[..., 8])
            if deg > 2:
                res = (res + _C3[0] * y * (3 * xx - yy) * sh[..., 9] + _C3[1] * xy * z * sh[..., 10] +
                       _C3[2] * y * (4 * zz - xx - yy) * sh[..., 11] +
                       _C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[..., 12] +
                       _C3[4] * x * (4 * zz - xx - yy) * sh[..., 13] + _C3[5] * z * (xx - yy) * sh[..., 14] +
                       _C3[6] * x * (xx - 3 * yy) * sh[..., 15])
    return res


def _prep_torch(pc, light, campos, wvt, sky_sh, sky_sh_degree, specular, fix_sky):
    """render()'s per-Gaussian steps as the reference writes them in PyTorch
    (gaussian_renderer/__init__.py:120-200; get_normal gaussian_model.py:115-122,
    build_rotation / get_minimum_axis / flip_align_view general_utils.py:98-170, get_depth
    gaussian_model.py:125-130), around the drop-in shade.  Returns [P, 14] rows in the
    column layout of relit_shade.relit_features."""
    import relit_shade
    xyz = pc.get_xyz
    d = xyz - campos[None]
    dirn = d / torch.sqrt(torch.clamp((d * d).sum(-1, keepdim=True), min=1e-20))
    q = pc.get_rotation
    q = q / torch.sqrt((q * q).sum(1, keepdim=True))
    r, x, y, z = q.unbind(1)
    R = torch.stack([torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], -1),
                     torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], -1),
                     torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1)], 1)
    axis = R.gather(2, pc.get_scaling.min(dim=-1)[1][..., None, None].expand(-1, 3, -1)).squeeze(2)
    n = axis * torch.where((axis * -dirn).sum(-1, keepdim=True) >= 0, 1, -1)
    is_sky = pc.get_is_sky.squeeze()
    fg = ~is_sky
    P = xyz.shape[0]
    rgb, ex = relit_shade.shade(light, xyz[fg][None, None], n[fg][None, None], pc.get_albedo[None, None],
                                campos.expand(int(fg.sum()), 3)[None, None], pc.get_roughness[None, None],
                                pc.get_metalness[None, None], specular=specular)
    cols = torch.zeros(P, 3, device=xyz.device)
    cols[fg] = rgb[0, 0]
    if fix_sky or sky_sh is None:
        cols[is_sky] = 1.0
    else:
        sh = sky_sh.transpose(1, 2)  # [1, 3, K] (coefficients last, as eval_sh takes them)
        cols[is_sky] = torch.clamp_min(eval_sh(sky_sh_degree, sh, dirn[is_sky]) + 0.5, 0.0)
    dif = torch.zeros(P, 3, device=xyz.device)
    dif[fg] = ex["diffuse"][0, 0]
    spe = torch.zeros(P, 3, device=xyz.device)
    spe[fg] = ex["specular"][0, 0]
    depth = torch.matmul(wvt.transpose(0, 1), torch.cat([xyz, torch.ones_like(xyz[:, :1])], -1).unsqueeze(-1))[:, 2]
    return torch.cat([cols, dif, spe, depth, 0.5 * n + 0.5, torch.ones(P, 1, device=xyz.device)], 1), is_sky


def render_calls(viewpoint_camera, pc, envlight, sky_sh, sky_sh_degree, pipe, bg_color, scaling_modifier=1.0,
                 debug=True, specular=True, fix_sky=False, normal_view=False):
    """render() as the reference sequences it: the per-Gaussian steps in PyTorch (around the
    drop-in shade) and one drop-in rasterizer call per image (the geometry cache makes the
    repeated calls colour-only).  Same arguments and outputs as `render`; the unfused
    baseline it is measured against (bench.py --config cfg3)."""
    import diff_gaussian_rasterization as dgr
    xyz = pc.get_xyz
    dev = xyz.device
    sp = torch.zeros_like(xyz, dtype=xyz.dtype, requires_grad=True) + 0
    try:
        sp.retain_grad()
    except Exception:
        pass
    st = dgr.GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
        tanfovx=math.tan(viewpoint_camera.FoVx * 0.5), tanfovy=math.tan(viewpoint_camera.FoVy * 0.5), bg=bg_color,
        scale_modifier=scaling_modifier, viewmatrix=viewpoint_camera.world_view_transform,
        projmatrix=viewpoint_camera.full_proj_transform, sh_degree=-1, campos=viewpoint_camera.camera_center,
        prefiltered=False)
    kw = dict(cov3D_precomp=pc.get_covariance(scaling_modifier)) if pipe.compute_cov3D_python else \
        dict(scales=pc.get_scaling, rotations=pc.get_rotation)
    f, is_sky = _prep_torch(pc, envlight, viewpoint_camera.camera_center, viewpoint_camera.world_view_transform,
                            sky_sh, sky_sh_degree, specular, fix_sky)
    rast = dgr.GaussianRasterizer(st)
    call = lambda col, r=rast: r(means3D=xyz, means2D=sp, shs=None, colors_precomp=col.contiguous(),
                                 opacities=pc.get_opacity, **kw)
    img, radii = call(f[:, 0:3])
    out = {"render": img, "viewspace_points": sp, "visibility_filter": radii > 0, "radii": radii}
    extras = {"diffuse_color": f[:, 3:6], "specular_color": f[:, 6:9], "depth": f[:, 9:10].repeat(1, 3),
              "normal": f[:, 10:13]}
    if debug:
        P = xyz.shape[0]
        fg = ~is_sky
        r_all = torch.zeros((P, 1), device=dev)
        r_all[fg] = pc.get_roughness
        m_all = torch.zeros((P, 1), device=dev)
        m_all[fg] = pc.get_metalness
        a_all = torch.ones_like(xyz)
        a_all[fg] = pc.get_albedo
        extras.update({"sky_color": f[:, 0:3] * is_sky[:, None].float(), "roughness": r_all.repeat(1, 3),
                       "metalness": m_all.repeat(1, 3), "albedo": a_all})
    sky_mask = viewpoint_camera.sky_mask.to(dev).squeeze()
    for k, v in extras.items():
        im = call(v)[0]
        if k == "normal":
            im = (im - 0.5) * 2.
            if normal_view:
                im = -im.clone()
            im = im * sky_mask + torch.ones_like(im) * (1 - sky_mask)
        out[k] = im
    ra = dgr.GaussianRasterizer(st._replace(bg=torch.zeros(3, device=dev)))
    out["alpha"] = call(torch.ones_like(xyz), ra)[0]
    nr = depth_to_normal(viewpoint_camera, (out["depth"][0] * sky_mask).unsqueeze(0)).permute(2, 0, 1)
    nr = nr * out["alpha"].detach()
    out["normal_ref"] = nr + torch.ones_like(nr) * (1 - sky_mask)
    return out
