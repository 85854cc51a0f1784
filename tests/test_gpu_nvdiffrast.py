"""nvdiffrast.torch.texture drop-in (csrc/gsr_texture.hip via gsr_texture2d_*) against the
oracle's restatement (orc_texture2d): forward, uv gradient and tex gradient, every
filter/boundary mode this build supports, broadcast and per-batch textures, plus the
reference's own call -- the split-sum FG LUT at light.py:170 (tex [1,256,256,2], uv
[1,1,N,2], linear/clamp) -- at the edges and in the interior of the LUT."""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _run(tex, uv, filt, boundary, dout):
    import nvdiffrast.torch as dr
    t = torch.from_numpy(tex).cuda().requires_grad_(True)
    u = torch.from_numpy(uv).cuda().requires_grad_(True)
    out = dr.texture(t, u, filter_mode=filt, boundary_mode=boundary)
    out.backward(torch.from_numpy(dout).cuda())
    return out.detach().cpu().numpy(), u.grad.cpu().numpy(), t.grad.cpu().numpy()


@pytest.mark.parametrize("filt", ["linear", "nearest"])
@pytest.mark.parametrize("boundary", ["clamp", "wrap", "zero"])
@pytest.mark.parametrize("tnb", [1, 2])
def test_texture_matches_oracle(filt, boundary, tnb):
    rng = np.random.default_rng(3)
    tex = rng.normal(0, 1, (tnb, 13, 17, 3)).astype(np.float32)
    uv = rng.uniform(-0.5, 1.5, (2, 9, 31, 2)).astype(np.float32)
    dout = rng.normal(0, 1, (2, 9, 31, 3)).astype(np.float32)
    out, d_uv, d_tex = _run(tex, uv, filt, boundary, dout)
    w_out, w_uv, w_tex = orc.texture2d(tex, uv, filt, boundary, dout=dout)
    # same operation order, no FMA contraction on either side: bit-identical
    np.testing.assert_array_equal(out, w_out)
    np.testing.assert_array_equal(d_uv, w_uv)
    np.testing.assert_allclose(d_tex, w_tex, rtol=1e-5, atol=2e-5)  # atomic summation order


def test_fg_lut_lookup_edges_and_interior():
    """light.py:168-170: fg_uv = (NdotV, roughness) with NdotV clamped >= 1e-4 and roughness
    in (0, 1); lookups on and beyond the edge texel centres and in the interior."""
    from gsr import assets
    lut = assets.load_fg_lut().reshape(1, 256, 256, 2).astype(np.float32)
    edge = np.array([0.0, 1e-4, 0.5 / 256, 0.5 / 256 + 1e-6, 1.0 / 256, 255.5 / 256, 0.999, 1.0, 1.01], np.float32)
    uu, vv = np.meshgrid(edge, edge)
    rng = np.random.default_rng(4)
    inner = rng.uniform(0.002, 0.998, (4000, 2)).astype(np.float32)
    uv = np.concatenate([np.stack([uu.ravel(), vv.ravel()], -1), inner])[None, None]
    dout = rng.normal(0, 1, uv.shape[:3] + (2,)).astype(np.float32)
    out, d_uv, _ = _run(lut, uv, "linear", "clamp", dout)
    w_out, w_uv, _ = orc.texture2d(lut, uv, "linear", "clamp", dout=dout)
    np.testing.assert_array_equal(out, w_out)
    np.testing.assert_array_equal(d_uv, w_uv)
    # texel (0, 0) = (0.009727, 0.990249) is what the corner returns
    np.testing.assert_allclose(out[0, 0, 0], lut[0, 0, 0], rtol=0, atol=0)


def test_texture_empty_and_validation():
    import nvdiffrast.torch as dr
    t = torch.zeros(1, 4, 4, 2, device="cuda")
    assert dr.texture(t, torch.zeros(1, 0, 5, 2, device="cuda"), filter_mode="linear").shape == (1, 0, 5, 2)
    with pytest.raises(ValueError):
        dr.texture(torch.zeros(3, 4, 4, 2, device="cuda"), torch.zeros(2, 1, 1, 2, device="cuda"))
