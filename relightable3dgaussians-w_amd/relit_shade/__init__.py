"""relit_shade -- drop-in HIP replacement for the per-Gaussian relighting shade.

Reference: scene/NVDIFFREC/light.py:131-193 EnvironmentLight.shade (+ utils/sh_utils.py
eval_sh / gauss_kernel / gamma_correction, scene/NVDIFFREC/util.py vector helpers and the
nvdiffrast LUT fetch).  The reference evaluates it as ~60-100 PyTorch kernels each way
with N x 25 x 3 intermediates; here it is one fused gfx950 kernel per direction
(libgsr.so: gsr_shade_forward / gsr_shade_backward), wrapped in an autograd Function.

Use either
  * `EnvironmentLight` from this module (same constructor / attributes / shade signature), or
  * `install(scene.NVDIFFREC.light.EnvironmentLight)` to route the reference class's
    `shade` method through the HIP op without touching caller code.
"""
import os
import sys

import numpy as np
import torch

_here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _here not in sys.path:
    sys.path.insert(0, _here)

from gsr import _lib, assets  # noqa: E402

__all__ = ["EnvironmentLight", "ShadeFunction", "shade", "install", "fg_lut", "relit_features", "RELIT_CHANNELS"]

_LUT = {}


def fg_lut(device):
    """The split-sum FG LUT [256,256,2] on `device` (light.py:41), sha256-checked."""
    key = str(device)
    if key not in _LUT:
        _LUT[key] = torch.from_numpy(assets.load_fg_lut()).to(device).contiguous()
    return _LUT[key]


def _flat3(t):
    return t.reshape(-1, 3).float().contiguous()


def _flat1(t):
    return None if t is None else t.reshape(-1).float().contiguous()


class ShadeFunction(torch.autograd.Function):
    """(pos, normal, albedo, view_pos [N,3], kr [N], km [N] | None, base [K,3]) ->
    (rgb, diffuse, specular) [N,3]."""

    @staticmethod
    def forward(ctx, pos, normal, albedo, view_pos, kr, km, base, lut, deg, specular):
        N = pos.shape[0]
        dev = pos.device
        rgb = torch.empty((N, 3), dtype=torch.float32, device=dev)
        dif = torch.empty_like(rgb)
        spe = torch.empty_like(rgb)
        if N:
            _lib.check(_lib.lib().gsr_shade_forward(
                N, deg, pos.data_ptr(), normal.data_ptr(), albedo.data_ptr(), view_pos.data_ptr(), kr.data_ptr(),
                None if km is None else km.data_ptr(), base.data_ptr(), lut.data_ptr(), int(specular),
                rgb.data_ptr(), dif.data_ptr(), spe.data_ptr(), _lib.stream_of(dev)), "gsr_shade_forward")
        ctx.deg, ctx.specular, ctx.has_km = deg, specular, km is not None
        ctx.save_for_backward(pos, normal, albedo, view_pos, kr, km if km is not None else kr, base, lut)
        return rgb, dif, spe

    @staticmethod
    def backward(ctx, g_rgb, g_dif, g_spe):
        pos, normal, albedo, view_pos, kr, km, base, lut = ctx.saved_tensors
        km = km if ctx.has_km else None
        N = pos.shape[0]
        dev = pos.device
        need = ctx.needs_input_grad
        out = lambda flag, like: torch.empty_like(like) if flag else None
        d_pos, d_n, d_a, d_vp = out(need[0], pos), out(need[1], normal), out(need[2], albedo), out(need[3], view_pos)
        d_kr = out(need[4], kr)
        d_km = out(need[5] and km is not None, kr)
        d_base = out(need[6], base)
        ws = None
        if d_base is not None:
            ws = torch.empty(int(_lib.lib().gsr_shade_workspace_bytes(N, ctx.deg)), dtype=torch.uint8, device=dev)
        c = lambda t: None if t is None else t.float().contiguous()
        g_rgb, g_dif, g_spe = c(g_rgb), c(g_dif), c(g_spe)
        ptr = lambda t: None if t is None else t.data_ptr()
        _lib.check(_lib.lib().gsr_shade_backward(
            N, ctx.deg, pos.data_ptr(), normal.data_ptr(), albedo.data_ptr(), view_pos.data_ptr(), kr.data_ptr(),
            ptr(km), base.data_ptr(), lut.data_ptr(), int(ctx.specular), ptr(g_rgb), ptr(g_dif),
            ptr(g_spe) if ctx.specular else None, ptr(d_pos), ptr(d_n), ptr(d_a), ptr(d_vp), ptr(d_kr), ptr(d_km),
            ptr(d_base), ptr(ws), _lib.stream_of(dev)), "gsr_shade_backward")
        return d_pos, d_n, d_a, d_vp, d_kr, d_km, d_base, None, None, None


def shade(light, gb_pos, gb_normal, albedo, view_pos, kr=None, km=None, specular=True):
    """EnvironmentLight.shade (light.py:131-193) on the HIP op.  Inputs [1,1,N,3] (kr, km
    [1,1,N,1]); returns (rgb [1,1,N,3], {"diffuse": ..., "specular": ...})."""
    _lib.require_gpu_tensor(gb_pos, "gb_pos")
    lead = albedo.shape[:-1]
    base = light.base.squeeze().reshape(-1, 3).float().contiguous()
    deg = int(round(base.shape[0] ** 0.5)) - 1
    if (deg + 1) ** 2 != base.shape[0]:
        raise ValueError(f"base has {base.shape[0]} SH coefficients, not a square")
    N = albedo.reshape(-1, 3).shape[0]
    if kr is None:
        if specular:
            raise ValueError("specular shading needs roughness kr")
        kr_ = torch.zeros(N, device=gb_pos.device)
    else:
        kr_ = _flat1(kr)
    rgb, dif, spe = ShadeFunction.apply(_flat3(gb_pos), _flat3(gb_normal), _flat3(albedo), _flat3(view_pos), kr_,
                                        _flat1(km), base, fg_lut(gb_pos.device), deg, bool(specular))
    rgb = rgb.reshape(*lead, 3)
    dif = dif.reshape(*lead, 3)
    if not specular:
        return dif, {"diffuse": dif, "specular": torch.zeros_like(dif)}
    return rgb, {"diffuse": dif, "specular": spe.reshape(*lead, 3)}


# column layout of relit_features rows (RELIT_STRIDE = 16 floats, the last two zero)
RELIT_CHANNELS = {"render": (0, 3), "diffuse_color": (3, 6), "specular_color": (6, 9), "depth": (9, 10),
                  "normal": (10, 13), "alpha": (13, 14)}


class RelitFeaturesFunction(torch.autograd.Function):
    """gsr_relit_features: render()'s per-Gaussian channels as [P, 16] feature rows."""

    @staticmethod
    def forward(ctx, xyz, rotation, scaling, albedo, roughness, metalness, base, sky_sh, fg_rank, fg_rows, campos,
                viewmatrix, lut, deg, sky_deg, specular, sink_in=None):
        P, N = xyz.shape[0], fg_rows.shape[0]
        dev = xyz.device
        feat = torch.empty((P, 16), dtype=torch.float32, device=dev)
        ws = torch.empty(int(_lib.lib().gsr_relit_workspace_bytes(P, N, deg, sky_deg)), dtype=torch.uint8, device=dev)
        ptr = lambda t: None if t is None or t.numel() == 0 else t.data_ptr()
        if P:
            _lib.check(_lib.lib().gsr_relit_features(
                P, N, xyz.data_ptr(), rotation.data_ptr(), scaling.data_ptr(), fg_rank.data_ptr(), ptr(fg_rows),
                ptr(albedo), ptr(roughness), ptr(metalness), deg, base.data_ptr(), lut.data_ptr(), int(specular),
                sky_deg, ptr(sky_sh), campos.data_ptr(), viewmatrix.data_ptr(), feat.data_ptr(), ws.data_ptr(),
                _lib.stream_of(dev)), "gsr_relit_features")
        ctx.deg, ctx.sky_deg, ctx.specular = deg, sky_deg, specular
        ctx.has = (roughness is not None, metalness is not None, sky_sh is not None)
        e = torch.empty(0, device=dev)
        ctx.save_for_backward(xyz, rotation, scaling, albedo, roughness if roughness is not None else e,
                              metalness if metalness is not None else e, base, sky_sh if sky_sh is not None else e,
                              fg_rank, fg_rows, campos, viewmatrix, lut, ws)
        # the model's tensors as render() passed them (xyz, rotation, albedo, roughness,
        # metalness): a training step's gsr.sink collects their gradients
        ctx.sink_in = sink_in
        return feat

    @staticmethod
    def backward(ctx, g_feat):
        (xyz, rotation, scaling, albedo, roughness, metalness, base, sky_sh, fg_rank, fg_rows, campos, viewmatrix, lut,
         ws) = ctx.saved_tensors
        P, N = xyz.shape[0], fg_rows.shape[0]
        dev = xyz.device
        from gsr import sink as gsink
        g_feat = g_feat.float().contiguous()
        need = ctx.needs_input_grad
        # gradients a training step's sink collects are added into its buffers by the kernels
        # (d_kr / d_km are written only with specular)
        sin = ctx.sink_in or (None,) * 5
        outs, ret, sk, claimed, acc = gsink.outputs(
            sin, (need[0], need[1], need[3] and albedo.numel() > 0, need[4] and ctx.specular and ctx.has[0],
                  need[5] and ctx.specular and ctx.has[1]))
        flat = lambda b: None if b is None else b.view(-1)
        d_xyz = outs[0] if outs[0] is not None else torch.empty_like(xyz)
        d_rot = outs[1] if outs[1] is not None else torch.empty_like(rotation)
        d_alb = outs[2] if outs[2] is not None else torch.empty_like(albedo)
        zk = torch.empty_like if ctx.specular else torch.zeros_like
        d_kr = flat(outs[3]) if outs[3] is not None else (zk(roughness) if ctx.has[0] else None)
        d_km = flat(outs[4]) if outs[4] is not None else (zk(metalness) if ctx.has[1] else None)
        d_base = torch.empty_like(base)
        d_sky = torch.empty_like(sky_sh) if ctx.has[2] and ctx.sky_deg >= 0 else None
        ptr = lambda t: None if t is None or t.numel() == 0 else t.data_ptr()
        _lib.check(_lib.lib().gsr_relit_features_backward(
            P, N, xyz.data_ptr(), rotation.data_ptr(), scaling.data_ptr(), fg_rank.data_ptr(), ptr(fg_rows),
            ptr(albedo), ptr(roughness), ptr(metalness), ctx.deg, base.data_ptr(), lut.data_ptr(), int(ctx.specular),
            ctx.sky_deg, ptr(sky_sh), campos.data_ptr(), viewmatrix.data_ptr(), g_feat.data_ptr(), d_xyz.data_ptr(),
            d_rot.data_ptr(), ptr(d_alb), ptr(d_kr), ptr(d_km), d_base.data_ptr(), ptr(d_sky), ws.data_ptr(), acc,
            _lib.stream_of(dev)), "gsr_relit_features_backward")
        if sk is not None:
            sk.done(claimed)
            keep = lambda g, i: None if outs[i] is not None else g
            d_xyz, d_rot, d_alb, d_kr, d_km = (keep(d_xyz, 0), keep(d_rot, 1), keep(d_alb, 2), keep(d_kr, 3),
                                               keep(d_km, 4))
        return (d_xyz, d_rot, None, d_alb, d_kr, d_km, d_base, d_sky, None, None, None, None, None, None, None, None,
                None)


_FG_CACHE = {}


def _fg_index(is_sky, P, dev):
    """(fg_rows, fg_rank) of the foreground Gaussians.  The sky flags change only when the
    model is densified, so the index (a nonzero: one host synchronisation) is cached on the
    flags' storage (address, shape, strides -- render() passes a fresh squeeze() view of the
    model's tensor every call) and version counter, and rebuilt when either changes.  The
    cache holds the flag tensor, so its storage cannot be freed and the address reused."""
    key = (is_sky.data_ptr(), tuple(is_sky.shape), tuple(is_sky.stride()), P, str(dev))
    hit = _FG_CACHE.get(key)
    if hit is not None and hit[1] == is_sky._version:
        return hit[2], hit[3]
    fg = ~is_sky.reshape(-1).bool()
    fg_rows = torch.nonzero(fg).reshape(-1).int()
    fg_rank = torch.full((P,), -1, dtype=torch.int32, device=dev)
    fg_rank[fg_rows.long()] = torch.arange(fg_rows.numel(), dtype=torch.int32, device=dev)
    if fg_rank.is_cuda:  # complete before another stream reads the cached index
        torch.cuda.current_stream(dev).synchronize()
    if len(_FG_CACHE) > 8:
        _FG_CACHE.clear()
    _FG_CACHE[key] = (is_sky, is_sky._version, fg_rows, fg_rank)
    return fg_rows, fg_rank


def relit_features(xyz, rotation, scaling, is_sky, albedo, roughness, metalness, light, campos, viewmatrix,
                   sky_sh=None, sky_sh_degree=1, specular=True, fix_sky=False):
    """render()'s per-Gaussian colour preparation (gaussian_renderer/__init__.py:120-200) as
    one fused op: returns features [P, 16] with the columns of RELIT_CHANNELS -- the shaded
    colour (sky colour for sky Gaussians), diffuse and specular (0 for sky), view-space
    depth, 0.5 normal + 0.5 and alpha = 1 -- ready for GaussianRasterizer.render_channels /
    rasterize_channels(nch=14).  Inputs as render() takes them from the model: xyz [P,3]
    (get_xyz), rotation [P,4] (get_rotation), scaling [P,3] (get_scaling), is_sky [P] or
    [P,1] bool, albedo [N_fg,3], roughness / metalness [N_fg,1], sky_sh [1, K, 3] (the
    sky SH; ignored with fix_sky), campos [3], viewmatrix = world_view_transform.
    Differentiable w.r.t. xyz, rotation, albedo, roughness, metalness, light.base, sky_sh."""
    _lib.require_gpu_tensor(xyz, "xyz")
    dev = xyz.device
    fg_rows, fg_rank = _fg_index(is_sky, xyz.shape[0], dev)
    base = light.base.squeeze().reshape(-1, 3).float().contiguous()
    deg = int(round(base.shape[0] ** 0.5)) - 1
    sky_deg = -1 if (fix_sky or sky_sh is None) else int(sky_sh_degree)
    sk = None
    if sky_deg >= 0:
        sk = sky_sh.reshape(-1, 3)
        if sk.shape[0] != (sky_deg + 1) ** 2:  # (a full-size slice would cost a zero tensor + copy backward)
            sk = sk[:(sky_deg + 1) ** 2]
        sk = sk.float().contiguous()
    from diff_gaussian_rasterization._C import _f32  # cached contiguous copies of camera matrices
    f = lambda t: None if t is None else t.float().contiguous()
    return RelitFeaturesFunction.apply(f(xyz), f(rotation), f(scaling), f(albedo), _flat1(roughness),
                                       _flat1(metalness), base, sk, fg_rank, fg_rows, _f32(campos), _f32(viewmatrix),
                                       fg_lut(dev), deg, sky_deg, bool(specular),
                                       (xyz, rotation, albedo, roughness, metalness))


class EnvironmentLight(torch.nn.Module):
    """Drop-in for scene/NVDIFFREC/light.py:14-193 EnvironmentLight (SH environment light,
    Ramamoorthi diffuse + split-sum specular); `shade` runs the fused HIP kernels."""

    C1, C2, C3, C4, C5 = 0.429043, 0.511664, 0.743125, 0.886227, 0.247708

    def __init__(self, base: torch.Tensor, sh_degree: int = 4):
        super().__init__()
        if sh_degree > 5:
            raise NotImplementedError
        self.sh_degree = sh_degree
        self.sh_dim = (sh_degree + 1) ** 2
        self.base = base.squeeze()
        self.NUM_CHANNELS = 3
        self._FG_LUT = fg_lut(base.device if base.is_cuda else "cuda").reshape(1, 256, 256, 2)

    def clone(self):
        return EnvironmentLight(self.base.clone().detach(), self.sh_degree)

    @property
    def get_shdim(self):
        return self.sh_dim

    @property
    def get_shdegree(self):
        return self.sh_degree

    @property
    def get_base(self):
        return self.base

    def set_base(self, base: torch.Tensor):
        assert base.squeeze().shape[0] == self.sh_dim, f"The number of SH coefficients must be {self.sh_dim}"
        self.base = base.squeeze()

    def get_diffuse_irradiance(self, normal):
        """light.py:65-94 (PyTorch; the shade itself uses the fused kernel)."""
        b = self.base
        x, y, z = normal[..., 0, None], normal[..., 1, None], normal[..., 2, None]
        return (self.C1 * b[8, :] * (x ** 2 - y ** 2) + self.C3 * b[6, :] * (z ** 2) + self.C4 * b[0, :] -
                self.C5 * b[6, :] + 2 * self.C1 * b[4, :] * x * y + 2 * self.C1 * b[7, :] * x * z +
                2 * self.C1 * b[5, :] * y * z + 2 * self.C2 * b[3, :] * x + 2 * self.C2 * b[1, :] * y +
                2 * self.C2 * b[2, :] * z)

    def get_specular_light_sh(self, kr):
        """light.py:97-119: gauss_kernel(kr) * base, [N, K, 3]."""
        l = torch.arange(self.sh_degree + 1, dtype=torch.float32, device=kr.device).view(1, -1)
        gl = torch.exp(-l * (l + 1) * (0.3 * kr))
        reps = torch.tensor([2 * i + 1 for i in range(self.sh_degree + 1)], device=kr.device)
        gw = torch.repeat_interleave(gl, reps, dim=1)
        return gw.unsqueeze(-1) * self.base.unsqueeze(0)

    def shade(self, gb_pos, gb_normal, albedo, view_pos, kr=None, km=None, specular=True):
        return shade(self, gb_pos, gb_normal, albedo, view_pos, kr, km, specular)


def install(light_cls):
    """Route `light_cls.shade` (e.g. scene.NVDIFFREC.light.EnvironmentLight) through the
    HIP op; the instance keeps its own `base`.  Returns the previous method."""
    prev = light_cls.shade

    def _shade(self, gb_pos, gb_normal, albedo, view_pos, kr=None, km=None, specular=True):
        return shade(self, gb_pos, gb_normal, albedo, view_pos, kr, km, specular)

    light_cls.shade = _shade
    return prev

