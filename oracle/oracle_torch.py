"""oracle/oracle_torch.py -- TEST INFRASTRUCTURE ONLY.

The C oracle (oracle/gsr_oracle.c) behind the reference's Python rasterizer API, on CPU
torch tensors: `GaussianRasterizationSettings`, `GaussianRasterizer` and
`rasterize_gaussians` with the argument order, validation and autograd gradient order of
`submodules/diff-gaussian-rasterization/diff_gaussian_rasterization/__init__.py:17-195`.

It exists so that tools/gen_golden_render.py can import the REFERENCE's own
`gaussian_renderer.render()` (gaussian_renderer/__init__.py:69-274) with this module
standing in for `diff_gaussian_rasterization` (SURVEY §8c recipe) and record render()'s
outputs and leaf gradients as fixtures.  Only tools/ and tests/ import it.
"""
from typing import NamedTuple

import numpy as np
import torch

from . import oracle as orc


class GaussianRasterizationSettings(NamedTuple):
    """diff_gaussian_rasterization/__init__.py:133-144 (same fields, same order)."""
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


import os

# GSR_ORACLE_VARIANT=f64: the rasterizer calls run the float64 build (exact-arithmetic proxy for
# tools/error_budget.py); their outputs are rounded to float32 as render() expects
F64 = os.environ.get("GSR_ORACLE_VARIANT", "") == "f64"


def _np(t):
    if t is None or (isinstance(t, torch.Tensor) and t.numel() == 0):
        return None
    return t.detach().cpu().contiguous().numpy().astype(np.float64 if F64 else np.float32)


class _OracleRasterize(torch.autograd.Function):
    """_RasterizeGaussians (__init__.py:42-131) over oracle.forward / oracle.backward."""

    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, st):
        bg = _np(st.bg)
        args = dict(bg=bg, means3D=_np(means3D), colors_precomp=_np(colors_precomp), scales=_np(scales),
                    rotations=_np(rotations), scale_modifier=float(st.scale_modifier), cov3D_precomp=_np(cov3Ds_precomp),
                    viewmatrix=_np(st.viewmatrix), projmatrix=_np(st.projmatrix), tanfovx=float(st.tanfovx),
                    tanfovy=float(st.tanfovy), sh=_np(sh), sh_degree=int(st.sh_degree), campos=_np(st.campos))
        fwd = orc.forward(opacities=_np(opacities), H=int(st.image_height), W=int(st.image_width),
                          prefiltered=bool(st.prefiltered), f64=F64, **args)
        ctx.fwd, ctx.args = fwd, args
        ctx.shapes = [None if t is None else t.shape for t in (means3D, sh, colors_precomp, opacities, scales,
                                                                rotations, cov3Ds_precomp)]
        color = torch.from_numpy(fwd["color"].astype(np.float32))
        radii = torch.from_numpy(fwd["radii"].copy())
        ctx.mark_non_differentiable(radii)
        return color, radii

    @staticmethod
    def backward(ctx, grad_color, _grad_radii):
        g = orc.backward(ctx.fwd, dL_dout=grad_color.detach().contiguous().numpy().astype(
            np.float64 if F64 else np.float32), f64=F64, **ctx.args)
        g = {k: (v.astype(np.float32) if isinstance(v, np.ndarray) and v.dtype == np.float64 else v)
             for k, v in g.items()}
        s_m3, s_sh, s_col, s_op, s_sc, s_rot, s_cov = ctx.shapes
        t = lambda a, shp: torch.from_numpy(np.ascontiguousarray(a)).reshape(shp) if shp is not None and \
            int(np.prod(shp)) > 0 else None
        # __init__.py:120-131: (means3D, means2D, sh, colors_precomp, opacities, scales,
        # rotations, cov3Ds_precomp, raster_settings)
        return (t(g["dL_dmeans3D"], s_m3), t(g["dL_dmean2D"], s_m3), t(g["dL_dsh"], s_sh),
                t(g["dL_dcolors"], s_col), t(g["dL_dopacity"], s_op), t(g["dL_dscales"], s_sc),
                t(g["dL_drotations"], s_rot), t(g["dL_dcov3D"], s_cov), None)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    return _OracleRasterize.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                                  raster_settings)


class GaussianRasterizer(torch.nn.Module):
    """__init__.py:146-195 (same validation and exception messages)."""

    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        with torch.no_grad():
            return torch.from_numpy(orc.mark_visible(_np(positions), _np(self.raster_settings.viewmatrix)))

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')
        e = torch.Tensor([])
        return rasterize_gaussians(means3D, means2D, e if shs is None else shs,
                                   e if colors_precomp is None else colors_precomp, opacities,
                                   e if scales is None else scales, e if rotations is None else rotations,
                                   e if cov3D_precomp is None else cov3D_precomp, self.raster_settings)
