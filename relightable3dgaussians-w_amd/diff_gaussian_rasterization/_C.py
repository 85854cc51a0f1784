"""diff_gaussian_rasterization._C -- the extension module the reference binds in
submodules/diff-gaussian-rasterization/ext.cpp:15-19, implemented over the C ABI of
libgsr.so (include/gsr.h) instead of a pybind11/libtorch extension.

Same three functions, same positional arguments and return tuples as
rasterize_points.h:18-64.  Every call runs the hand-written gfx950 kernels; there is no
CPU path (a CPU tensor raises).
"""
import ctypes as C
import os
import sys

import torch

_here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _here not in sys.path:
    sys.path.insert(0, _here)

from gsr import _lib  # noqa: E402

NUM_CHANNELS = 3


_SMALL = {}


def _f32(t):
    if t.dtype == torch.float32 and t.is_contiguous():
        return t
    if t.numel() <= 64:
        # camera matrices arrive transposed (scene/cameras.py:77, world_view_transform is a
        # .transpose(0, 1) view): their contiguous copy is cached per (storage, version,
        # layout, stream), so the six render() calls and each backward do not each launch a copy
        # kernel.  The cache holds the source, so its memory cannot be recycled into a false hit;
        # the stream is part of the key, so a hit is ordered after the copy that made it.
        stream = torch.cuda.current_stream(t.device).cuda_stream if t.is_cuda else 0
        key = (t.data_ptr(), t._version, tuple(t.shape), t.stride(), t.dtype, str(t.device), stream)
        hit = _SMALL.get(key)
        if hit is not None:
            return hit[1]
        c = t.float().contiguous()
        if len(_SMALL) >= 32:
            _SMALL.pop(next(iter(_SMALL)))
        _SMALL[key] = (t, c)
        return c
    return t.float().contiguous()


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                        viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                        prefiltered):
    """rasterize_points.cu:35-113 RasterizeGaussiansCUDA ->
    (num_rendered, color[3,H,W], radii[P] int32, geomBuffer, binningBuffer, imgBuffer)."""
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    _lib.require_gpu_tensor(means3D, "means3D")
    dev = means3D.device
    P, H, W = means3D.size(0), int(image_height), int(image_width)
    radii = torch.empty(P, dtype=torch.int32, device=dev)  # preprocess writes every entry (0 when culled)
    bs = _lib.BufferSet(dev)
    if P == 0:
        return 0, torch.zeros((NUM_CHANNELS, H, W), dtype=torch.float32, device=dev), radii, *bs.bufs
    out_color = torch.empty((NUM_CHANNELS, H, W), dtype=torch.float32, device=dev)
    M = sh.size(1) if sh.numel() != 0 and sh.size(0) != 0 else 0
    keep = [_f32(x) for x in (background, means3D, sh, colors, opacity, scales, rotations, cov3D_precomp, viewmatrix,
                              projmatrix, campos)]
    bg_, m_, sh_, col_, op_, sc_, rot_, cov_, vm_, pm_, cp_ = keep
    for name, t in (("background", bg_), ("viewmatrix", vm_), ("projmatrix", pm_), ("campos", cp_)):
        _lib.require_gpu_tensor(t, name)
    rc = _lib.ResizeContexts(bs)
    nr = C.c_int(0)
    try:
        ret = _lib.lib().gsr_forward(
            _lib.RESIZE, rc.ctx[0], _lib.RESIZE, rc.ctx[1], _lib.RESIZE, rc.ctx[2], P, int(degree), M,
            _lib.fptr(bg_), W, H, _lib.fptr(m_), _lib.fptr(sh_), _lib.fptr(col_), _lib.fptr(op_), _lib.fptr(sc_),
            float(scale_modifier), _lib.fptr(rot_), _lib.fptr(cov_), _lib.fptr(vm_), _lib.fptr(pm_), _lib.fptr(cp_),
            float(tan_fovx), float(tan_fovy), int(bool(prefiltered)), out_color.data_ptr(), radii.data_ptr(),
            _lib.stream_of(dev), C.byref(nr))
    finally:
        rc.close()
    _lib.check(ret, "rasterize_gaussians")
    return int(nr.value), out_color, radii, bs.bufs[0], bs.bufs[1], bs.bufs[2]


def _rasterize_reuse(background, colors, image_height, image_width, src_geom, src_radii, R, binningBuffer,
                     imageBuffer):
    """Colours-only forward over the geometry of an earlier rasterize_gaussians call
    (gsr_forward_reuse): same outputs as a full call whose geometry inputs are unchanged.
    Returns (num_rendered, color, radii, geomBuffer, binningBuffer, imageBuffer); the binning
    and image buffers are the earlier call's (shared, read-only)."""
    _lib.require_gpu_tensor(colors, "colors_precomp")
    dev = colors.device
    P, H, W = src_radii.size(0), int(image_height), int(image_width)
    radii = torch.empty(P, dtype=torch.int32, device=dev)
    out_color = torch.empty((NUM_CHANNELS, H, W), dtype=torch.float32, device=dev)
    bs = _lib.BufferSet(dev)
    if P == 0:
        out_color.zero_()
        return 0, out_color, radii, bs.bufs[0], binningBuffer, imageBuffer
    bg_, col_ = _f32(background), _f32(colors)
    rc = _lib.ResizeContexts(bs)
    ptr = lambda t: t.data_ptr() if t.numel() else None
    try:
        ret = _lib.lib().gsr_forward_reuse(_lib.RESIZE, rc.ctx[0], src_geom.data_ptr(), src_radii.data_ptr(),
                                           ptr(binningBuffer), imageBuffer.data_ptr(), P, int(R), _lib.fptr(bg_), W, H,
                                           _lib.fptr(col_), out_color.data_ptr(), radii.data_ptr(),
                                           _lib.stream_of(dev))
    finally:
        rc.close()
    _lib.check(ret, "rasterize_gaussians (geometry reuse)")
    return int(R), out_color, radii, bs.bufs[0], binningBuffer, imageBuffer


def rasterize_gaussians_backward(background, means3D, radii, colors, scales, rotations, scale_modifier,
                                 cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, sh, degree,
                                 campos, geomBuffer, R, binningBuffer, imageBuffer, *, colors_grad=True,
                                 cov3D_grad=True):
    """rasterize_points.cu:115-192 RasterizeGaussiansBackwardCUDA -> (dL_dmeans2D, dL_dcolors,
    dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations).

    colors_grad / cov3D_grad (keyword-only, default True as in the reference): False skips
    storing dL_dcolors / dL_dcov3D (returned as None) -- the autograd node passes them for
    inputs that need no gradient (render()'s empty colors_precomp and cov3D_precomp)."""
    _lib.require_gpu_tensor(means3D, "means3D")
    dev = means3D.device
    P = means3D.size(0)
    H, W = dL_dout_color.size(1), dL_dout_color.size(2)
    M = sh.size(1) if sh.numel() != 0 and sh.size(0) != 0 else 0
    # one allocation for the eight outputs (views of one flat buffer: each is written in full,
    # and the allocator calls were the host-side cost of this call); the reference's
    # dL_dconic is never returned, so it is not computed (NULL)
    colors_grad, cov3D_grad = bool(colors_grad), bool(cov3D_grad)
    widths = (3, NUM_CHANNELS if colors_grad else 0, 1, 3, 6 if cov3D_grad else 0, 3 * M, 3, 4)
    flat = (torch.zeros if P == 0 else torch.empty)(P * sum(widths), dtype=torch.float32, device=dev)
    outs, o = [], 0
    for w in widths:
        outs.append(flat[o:o + P * w])
        o += P * w
    dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations = (
        outs[0].view(P, 3), outs[1].view(P, widths[1]), outs[2].view(P, 1), outs[3].view(P, 3),
        outs[4].view(P, widths[4]), outs[5].view(P, M, 3), outs[6].view(P, 3), outs[7].view(P, 4))
    if P != 0:
        keep = [_f32(x) for x in (background, means3D, sh, colors, scales, rotations, cov3D_precomp, viewmatrix,
                                  projmatrix, campos, dL_dout_color)]
        bg_, m_, sh_, col_, sc_, rot_, cov_, vm_, pm_, cp_, dout_ = keep
        radii_ = radii.contiguous()
        ptr = lambda t: t.data_ptr() if t.numel() else None
        ret = _lib.lib().gsr_backward(
            P, int(degree), M, int(R), _lib.fptr(bg_), W, H, _lib.fptr(m_), _lib.fptr(sh_), _lib.fptr(col_),
            _lib.fptr(sc_), float(scale_modifier), _lib.fptr(rot_), _lib.fptr(cov_), _lib.fptr(vm_), _lib.fptr(pm_),
            _lib.fptr(cp_), float(tan_fovx), float(tan_fovy), radii_.data_ptr(), ptr(geomBuffer), ptr(binningBuffer),
            ptr(imageBuffer), _lib.fptr(dout_), dL_dmeans2D.data_ptr(), None,
            dL_dopacity.data_ptr(), dL_dcolors.data_ptr() if colors_grad else None, dL_dmeans3D.data_ptr(),
            dL_dcov3D.data_ptr() if cov3D_grad else None,
            dL_dsh.data_ptr() if M else None, dL_dscales.data_ptr(), dL_drotations.data_ptr(), _lib.stream_of(dev))
        _lib.check(ret, "rasterize_gaussians_backward")
    return (dL_dmeans2D, dL_dcolors if colors_grad else None, dL_dopacity, dL_dmeans3D,
            dL_dcov3D if cov3D_grad else None, dL_dsh, dL_dscales, dL_drotations)


def pack_features(features, nch=None):
    """[P, C] per-Gaussian channels -> contiguous 16-B aligned [P, stride] float32 whose first
    nch (default C) columns are the channels, stride a multiple of 4 (the multi-channel tile
    passes read 16-B rows).  A tensor that already has that layout (e.g. the [P, 16] rows of
    relit_shade.relit_features with nch = 14) is used as is."""
    P, C = features.shape
    nch = C if nch is None else int(nch)
    if features.dtype == torch.float32 and features.is_contiguous() and C % 4 == 0 and C >= nch and \
            features.data_ptr() % 16 == 0:
        return features
    stride = (nch + 3) // 4 * 4
    out = torch.zeros((P, stride), dtype=torch.float32, device=features.device)
    out[:, :nch] = features[:, :nch]
    return out


def rasterize_gaussians_channels(background, means3D, features, opacity, scales, rotations, scale_modifier,
                                 cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width,
                                 campos, prefiltered, nch=None):
    """All channels of several same-geometry rasterizer calls in one composite
    (gsr_forward_channels): background [nch], features [P, nch] ->
    (num_rendered, out[nch,H,W], radii, geomBuffer, binningBuffer, imgBuffer, packed features)."""
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    _lib.require_gpu_tensor(means3D, "means3D")
    dev = means3D.device
    P, H, W = means3D.size(0), int(image_height), int(image_width)
    nch = features.size(1) if nch is None else int(nch)
    if features.size(0) != P or background.numel() != nch or features.size(1) < nch:
        raise ValueError(f"features must be [P, nch] and background [nch] (P={P}, features {tuple(features.shape)}, "
                         f"background {tuple(background.shape)})")
    radii = torch.empty(P, dtype=torch.int32, device=dev)  # preprocess writes every entry (0 when culled)
    bs = _lib.BufferSet(dev)
    feat = pack_features(features if features.dtype == torch.float32 else features.float(), nch)
    out = torch.empty((nch, H, W), dtype=torch.float32, device=dev)
    keep = [_f32(x) for x in (background, means3D, opacity, scales, rotations, cov3D_precomp, viewmatrix, projmatrix,
                              campos)]
    bg_, m_, op_, sc_, rot_, cov_, vm_, pm_, cp_ = keep
    for name, t in (("background", bg_), ("features", feat), ("viewmatrix", vm_), ("projmatrix", pm_),
                    ("campos", cp_)):
        _lib.require_gpu_tensor(t, name)
    rc = _lib.ResizeContexts(bs)
    nr = C.c_int(0)
    try:
        ret = _lib.lib().gsr_forward_channels(
            _lib.RESIZE, rc.ctx[0], _lib.RESIZE, rc.ctx[1], _lib.RESIZE, rc.ctx[2], P, nch, feat.size(1),
            _lib.fptr(feat), _lib.fptr(bg_), W, H, _lib.fptr(m_), _lib.fptr(op_), _lib.fptr(sc_),
            float(scale_modifier), _lib.fptr(rot_), _lib.fptr(cov_), _lib.fptr(vm_), _lib.fptr(pm_), _lib.fptr(cp_),
            float(tan_fovx), float(tan_fovy), int(bool(prefiltered)), out.data_ptr(), radii.data_ptr(),
            _lib.stream_of(dev), C.byref(nr))
    finally:
        rc.close()
    _lib.check(ret, "rasterize_gaussians_channels")
    return int(nr.value), out, radii, bs.bufs[0], bs.bufs[1], bs.bufs[2], feat


def rasterize_gaussians_channels_backward(background, means3D, radii, feat, nch, scales, rotations, scale_modifier,
                                          cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout, campos,
                                          geomBuffer, R, binningBuffer, imageBuffer, dst=None, accumulate=0):
    """Backward of rasterize_gaussians_channels (gsr_backward_channels) -> (dL_dmeans2D,
    dL_dfeatures [P, stride] (columns >= nch zero), dL_dopacity, dL_dmeans3D, dL_dcov3D
    (empty without cov3D_precomp), dL_dscales, dL_drotations).  dst: optional buffers for
    "means3D", "scales", "rotations", "opacity" written in place, added into where their bit
    (GSR_ACC_*) is set in `accumulate` (gsr.sink)."""
    _lib.require_gpu_tensor(means3D, "means3D")
    dev = means3D.device
    P = means3D.size(0)
    H, W = dL_dout.size(1), dL_dout.size(2)
    alloc = torch.zeros if P == 0 else torch.empty
    f = dict(dtype=torch.float32, device=dev)
    dst = dst or {}
    dL_dmeans2D = alloc((P, 3), **f)
    dL_dopacity = dst["opacity"] if "opacity" in dst else alloc((P, 1), **f)
    dL_dfeat = alloc((P, feat.size(1)), **f)
    dL_dmeans3D = dst["means3D"] if "means3D" in dst else alloc((P, 3), **f)
    has_cov = cov3D_precomp is not None and cov3D_precomp.numel() > 0
    dL_dcov3D = alloc((P, 6), **f) if has_cov else torch.empty(0, **f)
    dL_dscales = dst["scales"] if "scales" in dst else alloc((P, 3), **f)
    dL_drotations = dst["rotations"] if "rotations" in dst else alloc((P, 4), **f)
    if P != 0:
        keep = [_f32(x) for x in (background, means3D, scales, rotations, cov3D_precomp, viewmatrix, projmatrix,
                                  campos, dL_dout)]
        bg_, m_, sc_, rot_, cov_, vm_, pm_, cp_, dout_ = keep
        ptr = lambda t: t.data_ptr() if t.numel() else None
        ret = _lib.lib().gsr_backward_channels(
            P, int(nch), feat.size(1), _lib.fptr(feat), int(R), _lib.fptr(bg_), W, H, _lib.fptr(m_), _lib.fptr(sc_),
            float(scale_modifier), _lib.fptr(rot_), _lib.fptr(cov_), _lib.fptr(vm_), _lib.fptr(pm_), _lib.fptr(cp_),
            float(tan_fovx), float(tan_fovy), radii.contiguous().data_ptr(), ptr(geomBuffer), ptr(binningBuffer),
            ptr(imageBuffer), _lib.fptr(dout_), dL_dmeans2D.data_ptr(), None, dL_dopacity.data_ptr(),
            dL_dfeat.data_ptr(), dL_dmeans3D.data_ptr(), ptr(dL_dcov3D), dL_dscales.data_ptr(),
            dL_drotations.data_ptr(), int(accumulate), _lib.stream_of(dev))
        _lib.check(ret, "rasterize_gaussians_channels_backward")
    return (dL_dmeans2D, dL_dfeat, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dscales, dL_drotations)


def mark_visible(means3D, viewmatrix, projmatrix):
    """rasterize_points.cu:194-213 markVisible -> bool[P]."""
    _lib.require_gpu_tensor(means3D, "means3D")
    P = means3D.size(0)
    present = torch.zeros(P, dtype=torch.bool, device=means3D.device)
    if P != 0:
        m_, vm_, pm_ = _f32(means3D), _f32(viewmatrix), _f32(projmatrix)
        _lib.check(_lib.lib().gsr_mark_visible(P, m_.data_ptr(), vm_.data_ptr(), pm_.data_ptr(), present.data_ptr(),
                                               _lib.stream_of(means3D.device)), "mark_visible")
    return present
