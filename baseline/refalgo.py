"""ctypes front end of libgsr_refalgo.so: the reference rasterizer's stage structure in
plain HIP (baseline/refalgo.hip), the GPU baseline bench.py times next to libgsr.

Not the product and not the oracle: a measured denominator for "x times the reference
rasterizer on the same MI355X" (BASELINE.md §2).  Parity with the CPU oracle is tested in
tests/test_gpu_refalgo.py so the baseline is known to compute the same images/gradients.
"""
import ctypes as C
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libgsr_refalgo.so")
SYMBOLS = ("gsr_ref_create", "gsr_ref_destroy", "gsr_ref_last_error", "gsr_ref_forward", "gsr_ref_backward")
_lib = None


def build(jobs=8, arch="gfx950"):
    subprocess.check_call(["make", "-s", "-C", HERE, f"-j{jobs}", f"ARCH={arch}"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run baseline.refalgo.build()")
        # libgsr_refalgo links libgsr's preprocess objects; load it on its own
        L = C.CDLL(LIB_PATH, mode=C.RTLD_LOCAL)
        vp, i, f = C.c_void_p, C.c_int, C.c_float
        L.gsr_ref_create.restype = vp
        L.gsr_ref_destroy.argtypes = [vp]
        L.gsr_ref_last_error.argtypes = [vp]
        L.gsr_ref_last_error.restype = C.c_char_p
        L.gsr_ref_forward.argtypes = [vp, vp, i, i, i, vp, i, i, vp, vp, vp, vp, vp, f, vp, vp, vp, vp, vp, f, f,
                                      vp, vp, C.POINTER(C.c_int)]
        L.gsr_ref_forward.restype = i
        L.gsr_ref_backward.argtypes = [vp, vp, i, i, vp, vp, vp, vp, f, vp, vp, vp, vp, vp, f, f, vp, vp, vp, vp, vp,
                                       vp, vp, vp, vp, vp, vp]
        L.gsr_ref_backward.restype = i
        _lib = L
    return _lib


def _p(t):
    return None if t is None or t.numel() == 0 else t.data_ptr()


class RefAlgoRasterizer:
    """forward()/backward() with the reference's _C argument meaning (rasterize_points.h:18-60)."""

    def __init__(self):
        self.L = lib()
        self.ctx = self.L.gsr_ref_create()

    def __del__(self):
        if getattr(self, "ctx", None):
            self.L.gsr_ref_destroy(self.ctx)
            self.ctx = None

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what}: {self.L.gsr_ref_last_error(self.ctx).decode()}")

    def forward(self, bg, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
                projmatrix, tan_fovx, tan_fovy, H, W, sh, degree, campos):
        bg, means3D, colors, opacity, scales, rotations, cov3D_precomp, viewmatrix, projmatrix, sh, campos = (
            t.contiguous() for t in (bg, means3D, colors, opacity, scales, rotations, cov3D_precomp, viewmatrix,
                                     projmatrix, sh, campos))
        P = means3D.shape[0]
        dev = means3D.device
        M = sh.shape[1] if sh.numel() else 0
        color = torch.empty(3, H, W, device=dev)
        radii = torch.empty(P, dtype=torch.int32, device=dev)
        R = C.c_int(0)
        s = torch.cuda.current_stream(dev).cuda_stream
        self._check(self.L.gsr_ref_forward(self.ctx, s, P, degree, M, _p(bg), W, H, _p(means3D), _p(sh), _p(colors),
                                           _p(opacity), _p(scales), scale_modifier, _p(rotations),
                                           _p(cov3D_precomp), _p(viewmatrix), _p(projmatrix), _p(campos), tan_fovx,
                                           tan_fovy, color.data_ptr(), radii.data_ptr(), C.byref(R)), "gsr_ref_forward")
        return R.value, color, radii

    def backward(self, bg, means3D, radii, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix, projmatrix,
                 tan_fovx, tan_fovy, dL_dout, sh, degree, campos):
        bg, means3D, radii, scales, rotations, cov3D_precomp, viewmatrix, projmatrix, dL_dout, sh, campos = (
            t.contiguous() for t in (bg, means3D, radii, scales, rotations, cov3D_precomp, viewmatrix, projmatrix,
                                     dL_dout, sh, campos))
        P = means3D.shape[0]
        dev = means3D.device
        M = sh.shape[1] if sh.numel() else 0
        z = lambda *s: torch.empty(*s, device=dev)
        g = dict(dL_dmeans2D=z(P, 3), dL_dcolors=z(P, 3), dL_dopacity=z(P, 1), dL_dmeans3D=z(P, 3),
                 dL_dcov3D=z(P, 6), dL_dsh=z(P, max(M, 0), 3), dL_dscales=z(P, 3), dL_drotations=z(P, 4))
        conic = z(P, 4)
        has_sr = scales.numel() > 0
        s = torch.cuda.current_stream(dev).cuda_stream
        self._check(self.L.gsr_ref_backward(
            self.ctx, s, degree, M, _p(bg), _p(means3D), _p(sh), _p(scales), scale_modifier, _p(rotations),
            _p(cov3D_precomp), _p(viewmatrix), _p(projmatrix), _p(campos), tan_fovx, tan_fovy, radii.data_ptr(),
            dL_dout.data_ptr(), g["dL_dmeans2D"].data_ptr(), conic.data_ptr(),
            g["dL_dopacity"].data_ptr(), g["dL_dcolors"].data_ptr(), g["dL_dmeans3D"].data_ptr(),
            g["dL_dcov3D"].data_ptr(), _p(g["dL_dsh"]), g["dL_dscales"].data_ptr() if has_sr else None,
            g["dL_drotations"].data_ptr() if has_sr else None), "gsr_ref_backward")
        if not has_sr:
            g["dL_dscales"].zero_()
            g["dL_drotations"].zero_()
        return tuple(g[k] for k in ("dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh",
                                    "dL_dscales", "dL_drotations"))
