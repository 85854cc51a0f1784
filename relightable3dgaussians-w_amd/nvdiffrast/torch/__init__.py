"""nvdiffrast.torch -- `texture()` with nvdiffrast's signature, on hand-written gfx950 HIP
(gsr_texture2d_forward / gsr_texture2d_backward, csrc/gsr_texture.hip).

The reference's live path calls it once per shade: the split-sum FG LUT lookup
`dr.texture(self._FG_LUT, fg_uv, filter_mode='linear', boundary_mode='clamp')`
(scene/NVDIFFREC/light.py:170, tex [1,256,256,2], uv [1,1,N,2]).  util.py:117 uses the
default 'wrap' boundary on latlong maps.  Supported: 2D textures, filter_mode 'auto' (no
mips given -> 'linear'), 'linear', 'nearest'; boundary_mode 'wrap', 'clamp', 'zero';
gradients to uv and tex.  Cube maps and mip-mapping (util.py:134/150, only reached from
dead code in this repo's reference) raise NotImplementedError.  GPU tensors only; there is
no CPU path.
"""
import os
import sys

import torch

_here = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _here not in sys.path:
    sys.path.insert(0, _here)

from gsr import _lib  # noqa: E402

__all__ = ["texture"]

_FILTERS = {"nearest": 0, "linear": 1}
_BOUNDARIES = {"wrap": 0, "clamp": 1, "zero": 2}


class _Texture2D(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tex, uv, filter_id, boundary_id):
        nb, h, w, _ = uv.shape
        tnb, th, tw, C = tex.shape
        out = torch.empty((nb, h, w, C), dtype=torch.float32, device=uv.device)
        _lib.check(_lib.lib().gsr_texture2d_forward(nb, h * w, tnb, th, tw, C, tex.data_ptr(), uv.data_ptr(),
                                                    filter_id, boundary_id, out.data_ptr(),
                                                    _lib.stream_of(uv.device)), "nvdiffrast.torch.texture")
        ctx.save_for_backward(tex, uv)
        ctx.modes = (filter_id, boundary_id)
        return out

    @staticmethod
    def backward(ctx, dout):
        tex, uv = ctx.saved_tensors
        filter_id, boundary_id = ctx.modes
        nb, h, w, _ = uv.shape
        tnb, th, tw, C = tex.shape
        dout = dout.float().contiguous()
        d_uv = torch.empty_like(uv) if ctx.needs_input_grad[1] else None
        d_tex = torch.zeros_like(tex) if ctx.needs_input_grad[0] else None
        if d_uv is not None or d_tex is not None:
            _lib.check(_lib.lib().gsr_texture2d_backward(
                nb, h * w, tnb, th, tw, C, tex.data_ptr(), uv.data_ptr(), filter_id, boundary_id, dout.data_ptr(),
                None if d_uv is None else d_uv.data_ptr(), None if d_tex is None else d_tex.data_ptr(),
                _lib.stream_of(uv.device)), "nvdiffrast.torch.texture (backward)")
        return d_tex, d_uv, None, None


def texture(tex, uv, uv_da=None, mip_level_bias=None, mip=None, filter_mode="auto", boundary_mode="wrap",
            max_mip_level=None):
    """nvdiffrast.torch.texture: sample tex [minibatch|1, tex_h, tex_w, C] at uv
    [minibatch, h, w, 2] -> [minibatch, h, w, C]."""
    if filter_mode == "auto":
        filter_mode = "linear-mipmap-linear" if (uv_da is not None or mip_level_bias is not None) else "linear"
    if boundary_mode == "cube" or filter_mode not in _FILTERS or mip is not None or uv_da is not None or \
            mip_level_bias is not None:
        raise NotImplementedError(f"nvdiffrast.torch.texture: filter_mode={filter_mode!r} "
                                  f"boundary_mode={boundary_mode!r} with mips/cube maps is not supported on this "
                                  "build (2D linear/nearest with wrap/clamp/zero is)")
    if boundary_mode not in _BOUNDARIES:
        raise ValueError(f"invalid boundary_mode {boundary_mode!r}")
    _lib.require_gpu_tensor(tex, "tex")
    _lib.require_gpu_tensor(uv, "uv")
    if tex.dim() != 4 or uv.dim() != 4 or uv.shape[-1] != 2:
        raise ValueError("tex must be [minibatch, height, width, channels] and uv [minibatch, height, width, 2]")
    if tex.shape[0] not in (1, uv.shape[0]):
        raise ValueError("minibatch size mismatch between tex and uv")
    return _Texture2D.apply(tex.float().contiguous(), uv.float().contiguous(), _FILTERS[filter_mode],
                            _BOUNDARIES[boundary_mode])
