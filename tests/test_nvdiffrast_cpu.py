"""The nvdiffrast drop-in (relightable3dgaussians-w_amd/nvdiffrast) on the CPU side:

* the reference's own scene/NVDIFFREC/light.py imports unchanged through it, with stub
  modules only for the absent cv2 / imageio / skimage (plus device="cuda" -> CPU for a module-level
  default argument, general_utils.py:295, since the build container has no GPU) -- light.py:4 and util.py:13 do
  `import nvdiffrast.torch as dr`;
* the oracle's restatement of dr.texture (orc_texture2d) agrees with the torch
  restatement the shade goldens were generated with (tools/gen_golden.py), its uv gradient
  with float64 finite differences, and its tex gradient with the adjoint identity
  <d_tex, X> = <dout, texture(X, uv)> (the lookup is linear in the texture).
nvdiffrast itself is third-party and absent: parity with it is unpinned beyond these.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "relightable3dgaussians-w_amd")
REF = "/root/reference"

_IMPORT_LIGHT = r"""
import sys, types
sys.dont_write_bytecode = True
sys.path.insert(0, {pkg!r})
for name in ("cv2", "imageio", "imageio.v3", "skimage", "skimage.measure"):
    sys.modules[name] = types.ModuleType(name)
sys.modules["imageio"].v3 = sys.modules["imageio.v3"]
sys.modules["cv2"].INTER_CUBIC = 2
import torch
# no GPU in the build container: map the module-level device="cuda" factories to the CPU
for fn in ("zeros", "ones", "tensor", "as_tensor", "empty", "full"):
    real = getattr(torch, fn)
    def wrap(f):
        def g(*a, **k):
            if "cuda" in str(k.get("device", "")):
                k["device"] = "cpu"
            return f(*a, **k)
        return g
    setattr(torch, fn, wrap(real))
sys.path.insert(0, {ref!r})
scene = types.ModuleType("scene")
scene.__path__ = [{ref!r} + "/scene"]
sys.modules["scene"] = scene
import nvdiffrast.torch as dr
from scene.NVDIFFREC.light import EnvironmentLight
from scene.NVDIFFREC import util
import scene.NVDIFFREC.light as light
assert light.dr is dr and util.dr is dr, "light.py must bind this repo's nvdiffrast"
assert dr.__file__.startswith({pkg!r}), dr.__file__
print("OK", EnvironmentLight.__name__, dr.texture.__module__)
"""


@pytest.mark.skipif(not os.path.isdir(REF), reason="needs the reference checkout (build container only)")
def test_reference_light_py_imports_through_the_shim():
    code = _IMPORT_LIGHT.format(pkg=PKG, ref=REF)
    r = subprocess.run([sys.executable, "-c", code], cwd=REF, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "OK EnvironmentLight nvdiffrast.torch" in r.stdout


def test_texture_api_rejects_unsupported_modes():
    sys.path.insert(0, PKG)
    import nvdiffrast.torch as dr
    t = torch.zeros(1, 4, 4, 2)
    uv = torch.zeros(1, 1, 3, 2)
    with pytest.raises(NotImplementedError):
        dr.texture(t, uv, boundary_mode="cube")
    with pytest.raises(NotImplementedError):
        dr.texture(t, uv, mip=[t], filter_mode="linear-mipmap-linear")
    with pytest.raises(RuntimeError, match="GPU"):  # no CPU path
        dr.texture(t, uv, filter_mode="linear", boundary_mode="clamp")


def _uv(rng, n, lo=-0.3, hi=1.3):
    return rng.uniform(lo, hi, (1, 1, n, 2)).astype(np.float32)


def test_oracle_texture_matches_golden_generator_restatement():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from gen_golden import texture_linear_clamp
    rng = np.random.default_rng(0)
    tex = rng.normal(0, 1, (1, 32, 24, 2)).astype(np.float32)
    uv = _uv(rng, 4000)
    want = texture_linear_clamp(torch.from_numpy(tex), torch.from_numpy(uv)).numpy()
    got = orc.texture2d(tex, uv, "linear", "clamp")
    np.testing.assert_allclose(got, want, rtol=0, atol=2e-6)


@pytest.mark.parametrize("boundary", ["clamp", "wrap", "zero"])
def test_oracle_texture_uv_gradient_finite_differences(boundary):
    rng = np.random.default_rng(1)
    tex = rng.normal(0, 1, (1, 16, 20, 3))
    uv = rng.uniform(-0.4, 1.4, (1, 1, 500, 2))
    dout = rng.normal(0, 1, (1, 1, 500, 3))
    _, d_uv, _ = orc.texture2d(tex, uv, "linear", boundary, dout=dout, f64=True)
    eps = 1e-7
    for k in range(2):
        e = np.zeros_like(uv)
        e[..., k] = eps
        fd = ((orc.texture2d(tex, uv + e, "linear", boundary, f64=True) -
               orc.texture2d(tex, uv - e, "linear", boundary, f64=True)) * dout).sum(-1) / (2 * eps)
        # skip lookups within eps of a texel centre line (the bilinear kink) or a clamp edge
        s = uv[..., k] * (20 if k == 0 else 16) - 0.5
        if boundary == "wrap":
            s = (uv[..., k] - np.floor(uv[..., k])) * (20 if k == 0 else 16) - 0.5
        ok = np.abs(s - np.round(s)) > 1e-4
        np.testing.assert_allclose(d_uv[..., k][ok], fd[ok], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("filt,boundary", [("linear", "clamp"), ("linear", "wrap"), ("linear", "zero"),
                                           ("nearest", "clamp"), ("nearest", "wrap"), ("nearest", "zero")])
def test_oracle_texture_tex_gradient_is_the_adjoint(filt, boundary):
    rng = np.random.default_rng(2)
    tex = rng.normal(0, 1, (2, 8, 10, 2))
    uv = rng.uniform(-0.4, 1.4, (2, 3, 50, 2))
    dout = rng.normal(0, 1, (2, 3, 50, 2))
    _, _, d_tex = orc.texture2d(tex, uv, filt, boundary, dout=dout, f64=True)
    X = rng.normal(0, 1, tex.shape)
    lhs = (d_tex * X).sum()
    rhs = (dout * orc.texture2d(X, uv, filt, boundary, f64=True)).sum()
    assert abs(lhs - rhs) < 1e-9 * max(1.0, abs(rhs))
