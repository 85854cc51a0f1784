"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes/numpy front end of the C restatement in oracle/gsr_oracle.c (see its header
for what is pinned and what is "parity unpinned").  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product path never does.

The functions mirror the reference's call sequence:
  forward()  = rasterizer_impl.cu:198-336   (preprocess, scan, duplicate, sort, ranges, render)
  backward() = rasterizer_impl.cu:340-433   (render bwd, cov2D bwd, preprocess bwd)
with outputs in the layouts rasterize_points.cu:35-192 returns.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.path.join(_HERE, "_build")
_libs = {}

BLOCK = 16


def build():
    """Compile the C oracle (float and float64 variants) with oracle/Makefile."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


# float build used by every f32 call: "" = the canonical oracle; "gpuexp", "ulp1", "ulp2", "fma"
# = the error-budget variants of oracle/Makefile (tools/error_budget.py, tests/test_error_budget.py)
VARIANTS = ("", "gpuexp", "ulp1", "ulp2", "fma")
_variant = os.environ.get("GSR_ORACLE_VARIANT", "")
_variant = "" if _variant == "f64" else _variant  # "f64": oracle_torch runs the float64 build


def use_variant(name=""):
    """Route every later float oracle call to build `name` (see VARIANTS); returns the previous."""
    global _variant
    if name not in VARIANTS:
        raise ValueError(f"unknown oracle variant {name!r}")
    prev, _variant = _variant, name
    return prev


def _lib(f64=False):
    key = "f64" if f64 else "f32" + _variant
    if key not in _libs:
        path = os.path.join(_BUILD, "liboracle64.so" if f64 else
                            ("liboracle_%s.so" % _variant if _variant else "liboracle.so"))
        if not os.path.exists(path):
            build()
        _libs[key] = C.CDLL(path)
    return _libs[key]


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _arr(x, dt):
    if x is None:
        return None
    return np.ascontiguousarray(np.asarray(x, dtype=dt))


def _real(f64):
    return (np.float64, C.c_double) if f64 else (np.float32, C.c_float)


def grid_dims(W, H):
    return (W + BLOCK - 1) // BLOCK, (H + BLOCK - 1) // BLOCK


def higher_msb(n):
    L = _lib()
    L.orc_higher_msb.restype = C.c_uint32
    return int(L.orc_higher_msb(C.c_uint32(n)))


def preprocess(means3D, scales, rotations, opacities, shs, colors_precomp, cov3D_precomp, viewmatrix,
               projmatrix, campos, W, H, tanfovx, tanfovy, scale_modifier=1.0, sh_degree=0, prefiltered=False,
               f64=False):
    dt, creal = _real(f64)
    L = _lib(f64)
    means3D = _arr(means3D, dt)
    P = means3D.shape[0]
    shs = _arr(shs, dt) if shs is not None and np.asarray(shs).size else None
    M = 0 if shs is None else shs.reshape(P, -1, 3).shape[1]
    out = dict(
        radii=np.zeros(P, np.int32), means2D=np.zeros((P, 2), dt), depths=np.zeros(P, dt),
        cov3D=np.zeros((P, 6), dt), rgb=np.zeros((P, 3), dt), conic_opacity=np.zeros((P, 4), dt),
        clamped=np.zeros((P, 3), np.uint8), tiles_touched=np.zeros(P, np.uint32))
    args = [
        C.c_int(P), C.c_int(sh_degree), C.c_int(M), _p(means3D), _p(_arr(scales, dt)), creal(scale_modifier),
        _p(_arr(rotations, dt)), _p(_arr(opacities, dt)), _p(shs), _p(_arr(cov3D_precomp, dt)),
        _p(_arr(colors_precomp, dt)), _p(_arr(viewmatrix, dt)), _p(_arr(projmatrix, dt)), _p(_arr(campos, dt)),
        C.c_int(W), C.c_int(H), creal(tanfovx), creal(tanfovy), C.c_int(int(prefiltered)),
        _p(out["radii"]), _p(out["means2D"]), _p(out["depths"]), _p(out["cov3D"]), _p(out["rgb"]),
        _p(out["conic_opacity"]), _p(out["clamped"]), _p(out["tiles_touched"])]
    L.orc_preprocess.restype = C.c_int
    err = L.orc_preprocess(*args)
    if err:
        raise RuntimeError("Point is filtered although prefiltered is set. This shouldn't happen!")
    return out


def binning(geom, W, H, f64=False):
    L = _lib(f64)
    P = geom["radii"].shape[0]
    L.orc_num_rendered.restype = C.c_int64
    R = int(L.orc_num_rendered(C.c_int(P), _p(geom["tiles_touched"])))
    gx, gy = grid_dims(W, H)
    keys = np.zeros(max(R, 1), np.uint64)
    vals = np.zeros(max(R, 1), np.uint32)
    ranges = np.zeros((gx * gy, 2), np.uint32)
    L.orc_binning.restype = C.c_int64
    L.orc_binning(C.c_int(P), C.c_int(W), C.c_int(H), _p(geom["means2D"]), _p(geom["depths"]), _p(geom["radii"]),
                  _p(geom["tiles_touched"]), _p(keys), _p(vals), _p(ranges))
    return R, keys[:R], vals[:R], ranges


def render_fwd(ranges, point_list, means2D, features, conic_opacity, bg, W, H, tiles=None, f64=False):
    dt, _ = _real(f64)
    L = _lib(f64)
    out = np.zeros((3, H, W), dt)
    final_T = np.zeros(H * W, dt)
    n_contrib = np.zeros(H * W, np.uint32)
    tl = None if tiles is None else _arr(tiles, np.int32)
    L.orc_render_fwd(C.c_int(W), C.c_int(H), _p(_arr(ranges, np.uint32)), _p(_arr(point_list, np.uint32)),
                     _p(_arr(means2D, dt)), _p(_arr(features, dt)), _p(_arr(conic_opacity, dt)), _p(_arr(bg, dt)),
                     _p(out), _p(final_T), _p(n_contrib), _p(tl), C.c_int(0 if tl is None else tl.shape[0]))
    return out, final_T, n_contrib


def render_bwd(P, ranges, point_list, bg, means2D, conic_opacity, colors, final_T, n_contrib, dL_dpix, W, H,
               tiles=None, f64=False):
    dt, _ = _real(f64)
    L = _lib(f64)
    g = dict(dL_dmean2D=np.zeros((P, 3), dt), dL_dconic=np.zeros((P, 2, 2), dt), dL_dopacity=np.zeros((P, 1), dt),
             dL_dcolors=np.zeros((P, 3), dt))
    tl = None if tiles is None else _arr(tiles, np.int32)
    L.orc_render_bwd(C.c_int(P), C.c_int(W), C.c_int(H), _p(_arr(ranges, np.uint32)),
                     _p(_arr(point_list, np.uint32)), _p(_arr(bg, dt)), _p(_arr(means2D, dt)),
                     _p(_arr(conic_opacity, dt)), _p(_arr(colors, dt)), _p(_arr(final_T, dt)),
                     _p(_arr(n_contrib, np.uint32)), _p(_arr(dL_dpix, dt)), _p(g["dL_dmean2D"]), _p(g["dL_dconic"]),
                     _p(g["dL_dopacity"]), _p(g["dL_dcolors"]), _p(tl), C.c_int(0 if tl is None else tl.shape[0]))
    return g


def forward(bg, means3D, colors_precomp, opacities, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
            projmatrix, tanfovx, tanfovy, H, W, sh, sh_degree, campos, prefiltered=False, f64=False):
    """rasterize_points.cu:35-113 RasterizeGaussiansCUDA: returns a dict with the public
    outputs (num_rendered, color[3,H,W], radii[P]) and every intermediate."""
    dt, _ = _real(f64)
    means3D = _arr(means3D, dt)
    P = means3D.shape[0]
    empty = lambda a: a is None or np.asarray(a).size == 0
    sh = None if empty(sh) else _arr(sh, dt)
    colors_precomp = None if empty(colors_precomp) else _arr(colors_precomp, dt)
    cov3D_precomp = None if empty(cov3D_precomp) else _arr(cov3D_precomp, dt)
    scales = None if empty(scales) else _arr(scales, dt)
    rotations = None if empty(rotations) else _arr(rotations, dt)
    geom = preprocess(means3D, scales, rotations, _arr(opacities, dt).reshape(-1), sh, colors_precomp,
                      cov3D_precomp, viewmatrix, projmatrix, campos, W, H, tanfovx, tanfovy, scale_modifier,
                      sh_degree, prefiltered, f64)
    R, keys, vals, ranges = binning(geom, W, H, f64)
    feats = colors_precomp if colors_precomp is not None else geom["rgb"]
    color, final_T, n_contrib = render_fwd(ranges, vals, geom["means2D"], feats, geom["conic_opacity"], bg, W, H,
                                           f64=f64)
    res = dict(geom)
    res.update(num_rendered=R, color=color, keys=keys, point_list=vals, ranges=ranges, final_T=final_T,
               n_contrib=n_contrib, features=feats, cov3D_used=cov3D_precomp if cov3D_precomp is not None
               else geom["cov3D"])
    return res


def preprocess_bwd(fwd, means3D, sh, sh_degree, scales, rotations, scale_modifier, viewmatrix, projmatrix, W, H,
                   tanfovx, tanfovy, campos, dL_dmean2D, dL_dconic, dL_dcolor, f64=False):
    dt, creal = _real(f64)
    L = _lib(f64)
    means3D = _arr(means3D, dt)
    P = means3D.shape[0]
    empty = lambda a: a is None or np.asarray(a).size == 0
    sh = None if empty(sh) else _arr(sh, dt)
    M = 0 if sh is None else sh.reshape(P, -1, 3).shape[1]
    scales = None if empty(scales) else _arr(scales, dt)
    rotations = None if empty(rotations) else _arr(rotations, dt)
    g = dict(dL_dmeans3D=np.zeros((P, 3), dt), dL_dcov3D=np.zeros((P, 6), dt), dL_dsh=np.zeros((P, M, 3), dt),
             dL_dscales=np.zeros((P, 3), dt), dL_drotations=np.zeros((P, 4), dt))
    L.orc_preprocess_bwd(C.c_int(P), C.c_int(sh_degree), C.c_int(M), _p(means3D), _p(fwd["radii"]), _p(sh),
                         _p(fwd["clamped"]), _p(scales), _p(rotations), creal(scale_modifier),
                         _p(_arr(fwd["cov3D_used"], dt)), _p(_arr(viewmatrix, dt)), _p(_arr(projmatrix, dt)),
                         C.c_int(W), C.c_int(H), creal(tanfovx), creal(tanfovy), _p(_arr(campos, dt)),
                         _p(_arr(dL_dmean2D, dt)), _p(_arr(dL_dconic, dt)), _p(_arr(dL_dcolor, dt)),
                         _p(g["dL_dmeans3D"]), _p(g["dL_dcov3D"]), _p(g["dL_dsh"]), _p(g["dL_dscales"]),
                         _p(g["dL_drotations"]))
    return g


def backward(fwd, bg, means3D, colors_precomp, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
             projmatrix, tanfovx, tanfovy, dL_dout, sh, sh_degree, campos, f64=False):
    """rasterize_points.cu:115-192 RasterizeGaussiansBackwardCUDA: returns the 8 gradients
    (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales,
    dL_drotations) in a dict."""
    dt, _ = _real(f64)
    dL_dout = _arr(dL_dout, dt)
    H, W = dL_dout.shape[1], dL_dout.shape[2]
    P = np.asarray(means3D).shape[0]
    g = render_bwd(P, fwd["ranges"], fwd["point_list"], bg, fwd["means2D"], fwd["conic_opacity"], fwd["features"],
                   fwd["final_T"], fwd["n_contrib"], dL_dout, W, H, f64=f64)
    g2 = preprocess_bwd(fwd, means3D, sh, sh_degree, scales, rotations, scale_modifier, viewmatrix, projmatrix, W,
                        H, tanfovx, tanfovy, campos, g["dL_dmean2D"], g["dL_dconic"], g["dL_dcolors"], f64=f64)
    g.update(g2)
    return g


def mark_visible(means3D, viewmatrix, f64=False):
    dt, _ = _real(f64)
    means3D = _arr(means3D, dt)
    out = np.zeros(means3D.shape[0], np.uint8)
    _lib(f64).orc_mark_visible(C.c_int(means3D.shape[0]), _p(means3D), _p(_arr(viewmatrix, dt)), _p(out))
    return out.astype(bool)


def eval_sh(deg, sh, dirs, f64=False):
    """sh: [N, K, 3] (coefficient-major, as the shade's spec_light) ; dirs [N,3] -> [N,3]"""
    dt, _ = _real(f64)
    sh = _arr(sh, dt)
    dirs = _arr(dirs, dt)
    N, K = sh.shape[0], sh.shape[1]
    out = np.zeros((N, 3), dt)
    _lib(f64).orc_eval_sh(C.c_int(deg), C.c_int(N), _p(sh), C.c_int(K), _p(dirs), _p(out))
    return out


def shade_fwd(pos, nrm, albedo, view_pos, kr, km, base, lut, deg=4, specular=True, f64=False):
    dt, _ = _real(f64)
    N = np.asarray(pos).reshape(-1, 3).shape[0]
    a = [_arr(np.asarray(x).reshape(-1, 3), dt) for x in (pos, nrm, albedo, view_pos)]
    kr_ = _arr(np.asarray(kr).reshape(-1), dt)
    km_ = None if km is None else _arr(np.asarray(km).reshape(-1), dt)
    base_ = _arr(np.asarray(base).reshape(-1, 3), dt)
    lut_ = _arr(np.asarray(lut).reshape(256, 256, 2), dt)
    rgb, dif, spe = (np.zeros((N, 3), dt) for _ in range(3))
    _lib(f64).orc_shade_fwd(C.c_int(N), C.c_int(deg), *[_p(x) for x in a], _p(kr_), _p(km_), _p(base_), _p(lut_),
                            C.c_int(int(specular)), _p(rgb), _p(dif), _p(spe))
    return rgb, dif, spe


def shade_bwd(pos, nrm, albedo, view_pos, kr, km, base, lut, g_rgb, g_diff, g_spec, deg=4, specular=True,
              f64=False):
    dt, _ = _real(f64)
    N = np.asarray(pos).reshape(-1, 3).shape[0]
    a = [_arr(np.asarray(x).reshape(-1, 3), dt) for x in (pos, nrm, albedo, view_pos)]
    kr_ = _arr(np.asarray(kr).reshape(-1), dt)
    km_ = None if km is None else _arr(np.asarray(km).reshape(-1), dt)
    base_ = _arr(np.asarray(base).reshape(-1, 3), dt)
    lut_ = _arr(np.asarray(lut).reshape(256, 256, 2), dt)
    gs = [_arr(np.asarray(x).reshape(-1, 3), dt) for x in (g_rgb, g_diff, g_spec)]
    d = dict(pos=np.zeros((N, 3), dt), normal=np.zeros((N, 3), dt), albedo=np.zeros((N, 3), dt),
             view_pos=np.zeros((N, 3), dt), kr=np.zeros(N, dt), km=None if km is None else np.zeros(N, dt),
             base=np.zeros(base_.shape, dt))
    _lib(f64).orc_shade_bwd(C.c_int(N), C.c_int(deg), *[_p(x) for x in a], _p(kr_), _p(km_), _p(base_), _p(lut_),
                            C.c_int(int(specular)), *[_p(x) for x in gs], _p(d["pos"]), _p(d["normal"]),
                            _p(d["albedo"]), _p(d["view_pos"]), _p(d["kr"]), _p(d["km"]), _p(d["base"]))
    return d


def texture2d(tex, uv, filter_mode="linear", boundary_mode="clamp", dout=None, f64=False):
    """nvdiffrast dr.texture, 2D (orc_texture2d_fwd/bwd): tex [tnb,th,tw,C], uv [nb,h,w,2]
    -> out [nb,h,w,C]; with dout also (d_uv, d_tex)."""
    dt, _ = _real(f64)
    L = _lib(f64)
    tex = _arr(tex, dt)
    uv = _arr(uv, dt)
    tnb, th, tw, Cc = tex.shape
    nb, h, w, _ = uv.shape
    fm = {"nearest": 0, "linear": 1}[filter_mode]
    bm = {"wrap": 0, "clamp": 1, "zero": 2}[boundary_mode]
    args = [C.c_int(nb), C.c_int(h * w), C.c_int(tnb), C.c_int(th), C.c_int(tw), C.c_int(Cc), _p(tex), _p(uv),
            C.c_int(fm), C.c_int(bm)]
    out = np.zeros((nb, h, w, Cc), dt)
    L.orc_texture2d_fwd(*args, _p(out))
    if dout is None:
        return out
    d_uv = np.zeros_like(uv)
    d_tex = np.zeros_like(tex)
    L.orc_texture2d_bwd(*args, _p(_arr(dout, dt)), _p(d_uv), _p(d_tex))
    return out, d_uv, d_tex


def knn(points):
    """submodules/simple-knn distCUDA2: mean squared distance to the 3 nearest other points
    (orc_knn, the reference's Morton/box algorithm, float arithmetic)."""
    L = _lib(False)
    pts = _arr(points, np.float32).reshape(-1, 3)
    out = np.zeros(pts.shape[0], np.float32)
    L.orc_knn(C.c_int(pts.shape[0]), _p(pts), _p(out))
    return out
