"""Drop-in `diff_gaussian_rasterization` package for MI355X.

Public surface identical to the reference package
(submodules/diff-gaussian-rasterization/diff_gaussian_rasterization/__init__.py:17-195),
so gaussian_renderer/__init__.py:15 `from diff_gaussian_rasterization import
GaussianRasterizationSettings, GaussianRasterizer` and everything built on it run
unchanged.  The extension module `_C` is backed by libgsr.so (hand-written gfx950 HIP).
"""
import os
from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "_RasterizeGaussians",
           "geometry_cache", "rasterize_channels"]


class _GeometryCache:
    """Geometry reuse across rasterizer calls that differ only in colours.

    render() (gaussian_renderer/__init__.py:160-264) rasterizes the same Gaussians 6-10 times
    per view -- the main image, diffuse/specular/depth/normal extras and the alpha mask --
    with different colors_precomp and background.  Preprocess, depth sort, binning and the
    tile ranges depend only on the geometry, so a call whose geometry inputs are the same
    tensors, unmodified (data pointer, version counter, shape, strides), with the same camera
    and image settings, on the same HIP stream, re-renders colours over the previous call's binning
    (gsr_forward_reuse).  The outputs are bit-identical to a full call.  The cache holds
    references to the keyed tensors, so their memory cannot be recycled into a false hit
    while it lives.  Only the colors_precomp path is cached (SH colours depend on campos).
    Disable with GSR_GEOMETRY_CACHE=0 or geometry_cache(False)."""

    def __init__(self):
        self.enabled = os.environ.get("GSR_GEOMETRY_CACHE", "1") != "0"
        self.clear()

    def clear(self):
        self.key = None
        self.refs = None
        self.entry = None
        self.hits = 0
        self.misses = 0

    @staticmethod
    def _tkey(t):
        if t is None or t.numel() == 0:
            return None
        return (t.data_ptr(), t._version, tuple(t.shape), t.stride(), t.dtype, str(t.device))

    def key_of(self, s, means3D, opacities, scales, rotations, cov3Ds_precomp):
        """The key includes the current HIP stream: a hit reuses the miss call's binning and
        image buffers (and rewrites parts of the image buffer), which is ordered only on the
        stream that produced them.  A call on another stream misses."""
        tensors = (means3D, opacities, scales, rotations, cov3Ds_precomp, s.viewmatrix, s.projmatrix)
        stream = torch.cuda.current_stream(means3D.device).cuda_stream
        return (tuple(self._tkey(t) for t in tensors),
                (int(s.image_height), int(s.image_width), float(s.tanfovx), float(s.tanfovy),
                 float(s.scale_modifier), bool(s.prefiltered)), stream), tensors


_geometry_cache = _GeometryCache()


def geometry_cache(enabled=None):
    """Query or switch the geometry cache; returns the cache (hits/misses counters)."""
    if enabled is not None:
        _geometry_cache.enabled = bool(enabled)
        _geometry_cache.clear()
    return _geometry_cache


class GaussianRasterizationSettings(NamedTuple):
    """Camera + render settings (reference __init__.py:133-144).  viewmatrix is the
    camera's world_view_transform, projmatrix its full_proj_transform (row-vector
    convention, scene/cameras.py:77-79)."""
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings)


def _forward_args(s, means3D, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, sh):
    # positional order of _C.rasterize_gaussians (rasterize_points.h:18-37)
    return (s.bg, means3D, colors_precomp, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
            s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width, sh, s.sh_degree,
            s.campos, s.prefiltered)


class _RasterizeGaussians(torch.autograd.Function):
    """Autograd node (reference __init__.py:40-131).  means2D is an input only so that its
    .grad receives dL/d(screen-space mean) for densification; the forward never reads it."""

    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings):
        cache = _geometry_cache
        key = None
        if cache.enabled and colors_precomp.numel() != 0 and sh.numel() == 0 and means3D.is_cuda:
            key, refs = cache.key_of(raster_settings, means3D, opacities, scales, rotations, cov3Ds_precomp)
        if key is not None and key == cache.key:
            cache.hits += 1
            R0, radii0, geom0, bin0, img0 = cache.entry
            num_rendered, color, radii, geom_buf, bin_buf, img_buf = _C._rasterize_reuse(
                raster_settings.bg, colors_precomp, raster_settings.image_height, raster_settings.image_width, geom0,
                radii0, R0, bin0, img0)
        else:
            num_rendered, color, radii, geom_buf, bin_buf, img_buf = _C.rasterize_gaussians(
                *_forward_args(raster_settings, means3D, colors_precomp, opacities, scales, rotations,
                               cov3Ds_precomp, sh))
            if key is not None:
                cache.misses += 1
                cache.key, cache.refs = key, refs
                cache.entry = (num_rendered, radii, geom_buf, bin_buf, img_buf)
        ctx.raster_settings = raster_settings
        ctx.num_rendered = num_rendered
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geom_buf,
                              bin_buf, img_buf)
        return color, radii

    @staticmethod
    def backward(ctx, grad_out_color, _grad_radii):
        s = ctx.raster_settings
        colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geom_buf, bin_buf, img_buf = \
            ctx.saved_tensors
        (g_means2D, g_colors, g_opacities, g_means3D, g_cov3D, g_sh, g_scales, g_rotations) = \
            _C.rasterize_gaussians_backward(s.bg, means3D, radii, colors_precomp, scales, rotations,
                                            s.scale_modifier, cov3Ds_precomp, s.viewmatrix, s.projmatrix, s.tanfovx,
                                            s.tanfovy, grad_out_color, sh, s.sh_degree, s.campos, geom_buf,
                                            ctx.num_rendered, bin_buf, img_buf,
                                            colors_grad=ctx.needs_input_grad[3], cov3D_grad=ctx.needs_input_grad[7])
        # gradients in the order of forward()'s inputs; None for raster_settings (and for an empty
        # colors_precomp / cov3D_precomp, which need none: their 36 B per Gaussian are not stored)
        return g_means3D, g_means2D, g_sh, g_colors, g_opacities, g_scales, g_rotations, g_cov3D, None


# num_rendered (the reference's R, the sum of tiles touched) and the visible count of the latest
# multi-channel call, recorded only while record_channels_calls(True) is on (bench.py's training
# leg reads them for its algorithmic bytes); scalars, so no device tensor stays alive
last_channels_call = {"num_rendered": None, "visible": None, "enabled": False}


def record_channels_calls(on=True):
    """Turn the last_channels_call record on or off (off by default; the visible count costs
    one device reduction and a host sync per call while on)."""
    last_channels_call["enabled"] = bool(on)


def rasterize_channels(means3D, means2D, features, opacities, scales, rotations, cov3Ds_precomp, background,
                       raster_settings, nch=None):
    """Composite of the first nch (default all) per-Gaussian channels of `features` [P, C]
    over one geometry (gsr_forward_channels): returns (image [nch, H, W], radii).  Channel c
    equals the reference rasterizer's output for colours holding channel c with
    background[c]."""
    return _RasterizeChannels.apply(means3D, means2D, features, opacities, scales, rotations, cov3Ds_precomp,
                                    background, raster_settings, nch)


class _RasterizeChannels(torch.autograd.Function):
    """Autograd node of the multi-channel composite.  Gradients: features, the geometry
    inputs and means2D (summed over the channels, as autograd sums them over the separate
    calls render() makes); none for background (the reference returns none for bg)."""

    @staticmethod
    def forward(ctx, means3D, means2D, features, opacities, scales, rotations, cov3Ds_precomp, background,
                raster_settings, nch=None):
        s = raster_settings
        num_rendered, out, radii, geom_buf, bin_buf, img_buf, feat = _C.rasterize_gaussians_channels(
            background, means3D, features, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
            s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width, s.campos, s.prefiltered,
            nch)
        ctx.raster_settings = s
        ctx.num_rendered = num_rendered
        if last_channels_call["enabled"]:
            last_channels_call["num_rendered"] = num_rendered
            last_channels_call["visible"] = int((radii > 0).sum().item())
        ctx.nch = features.shape[1] if nch is None else int(nch)
        ctx.ncols = features.shape[1]
        ctx.save_for_backward(background, feat, means3D, scales, rotations, cov3Ds_precomp, radii, geom_buf, bin_buf,
                              img_buf)
        # inputs whose gradient a training step's gsr.sink collects (the kernels add into it)
        ctx.sink_in = (means3D, scales, rotations, opacities)
        return out, radii

    @staticmethod
    def backward(ctx, grad_out, _grad_radii):
        from gsr import sink as gsink
        s = ctx.raster_settings
        background, feat, means3D, scales, rotations, cov3Ds_precomp, radii, geom_buf, bin_buf, img_buf = \
            ctx.saved_tensors
        need = ctx.needs_input_grad
        keys = ("means3D", "scales", "rotations", "opacity")
        outs, ret, sk, claimed, acc = gsink.outputs(ctx.sink_in, (need[0], need[4], need[5], need[3]))
        dst = {k: o for k, o in zip(keys, outs) if o is not None}
        (g_means2D, g_feat, g_opacities, g_means3D, g_cov3D, g_scales, g_rotations) = \
            _C.rasterize_gaussians_channels_backward(background, means3D, radii, feat, ctx.nch, scales, rotations,
                                                     s.scale_modifier, cov3Ds_precomp, s.viewmatrix, s.projmatrix,
                                                     s.tanfovx, s.tanfovy, grad_out, s.campos, geom_buf,
                                                     ctx.num_rendered, bin_buf, img_buf, dst=dst, accumulate=acc)
        if sk is not None:
            sk.done(claimed)
            g_means3D, g_scales, g_rotations, g_opacities = (
                g if r else None for g, r in zip((g_means3D, g_scales, g_rotations, g_opacities), ret))
        if g_cov3D.numel() == 0:
            g_cov3D = None
        if g_feat.shape[1] >= ctx.ncols:  # gradient for every input column (columns >= nch: 0)
            g_feat = g_feat[:, :ctx.ncols]
        else:
            g_full = torch.zeros((g_feat.shape[0], ctx.ncols), dtype=g_feat.dtype, device=g_feat.device)
            g_full[:, :g_feat.shape[1]] = g_feat
            g_feat = g_full
        return g_means3D, g_means2D, g_feat, g_opacities, g_scales, g_rotations, g_cov3D, None, None, None


class GaussianRasterizer(nn.Module):
    """reference __init__.py:146-195"""

    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        with torch.no_grad():
            s = self.raster_settings
            return _C.mark_visible(positions, s.viewmatrix, s.projmatrix)

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        if (shs is None) == (colors_precomp is None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')
        empty = torch.Tensor([])
        pick = lambda t: empty if t is None else t
        return rasterize_gaussians(means3D, means2D, pick(shs), pick(colors_precomp), opacities, pick(scales),
                                   pick(rotations), pick(cov3D_precomp), self.raster_settings)

    def render_channels(self, means3D, means2D, opacities, colors, backgrounds=None, scales=None, rotations=None,
                        cov3D_precomp=None):
        """Several same-geometry rasterizations in one composite (the extension behind
        render()'s 6-10 calls).  colors: list of [P, k_i] tensors;
        backgrounds: list of [k_i] tensors (default: raster_settings.bg for 3-channel entries,
        zeros otherwise).  Returns ([image_i [k_i, H, W]], radii); image_i equals
        forward(colors_precomp=colors[i]) with that background, and gradients flow to every
        colour tensor and the geometry as through separate calls."""
        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')
        s = self.raster_settings
        ks = [int(c.shape[1]) for c in colors]
        if backgrounds is None:
            backgrounds = [None] * len(colors)
        bgs = []
        for k, b in zip(ks, backgrounds):
            if b is None:
                b = s.bg if (k == 3 and s.bg.numel() == 3) else torch.zeros(k, device=means3D.device)
            bgs.append(b.reshape(-1).float())
        empty = torch.Tensor([])
        pick = lambda t: empty if t is None else t
        out, radii = rasterize_channels(means3D, means2D, torch.cat([c.float() for c in colors], 1), opacities,
                                        pick(scales), pick(rotations), pick(cov3D_precomp), torch.cat(bgs), s)
        return list(torch.split(out, ks, 0)), radii
