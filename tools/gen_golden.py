"""Generate golden vectors by importing the REFERENCE's own Python (read-only at
/root/reference) on the CPU.  Output: tests/golden/*.npz (inputs + expected outputs only;
no reference source is stored).  Run in the build container:

    python tools/gen_golden.py

Pinned by these fixtures:
  eval_sh deg 0..5        utils/sh_utils.py:81-151
  gauss_kernel            utils/sh_utils.py:162-181
  EnvironmentLight.shade  scene/NVDIFFREC/light.py:131-193 (forward + autograd backward)
                          -- except nvdiffrast dr.texture, which is not vendored; the stub
                          below is this repo's restatement (parity unpinned for the LUT fetch)
  cov3D                   scene/gaussian_model.py:30-34 build_covariance_from_scaling_rotation
  depth                   scene/gaussian_model.py:125-130 get_depth
  normals                 scene/gaussian_model.py:115-122 get_normal (min-scale axis + flip)
  cameras                 utils/graphics_utils.py:47-80 + scene/cameras.py:74-79
  SH -> RGB (deg <= 3)    eval_sh + 0.5, clamp >= 0 (the rasterizer's computeColorFromSH,
                          forward.cu:20-71, uses the same polynomial and constants)
Stubs: cv2, imageio, skimage, plyfile, simple_knn, nvdiffrast (absent from this image);
device "cuda" is mapped to the CPU.  Nothing is executed from any serialized file.
"""
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def _stub(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def texture_linear_clamp(tex, uv, filter_mode="linear", boundary_mode="clamp"):
    """This repo's restatement of nvdiffrast.torch.texture for a [1,Ht,Wt,C] texture,
    uv [1,h,w,2], bilinear, clamp-to-edge, texel centres at (i+0.5)/size; u -> width."""
    assert filter_mode == "linear" and boundary_mode == "clamp"
    _, Ht, Wt, Cc = tex.shape
    u = uv[..., 0] * Wt - 0.5
    v = uv[..., 1] * Ht - 0.5
    x0f = torch.floor(u).detach()
    y0f = torch.floor(v).detach()
    fx = (u - x0f)[..., None]
    fy = (v - y0f)[..., None]
    x0 = x0f.long()
    y0 = y0f.long()
    x1 = (x0 + 1).clamp(0, Wt - 1)
    y1 = (y0 + 1).clamp(0, Ht - 1)
    x0 = x0.clamp(0, Wt - 1)
    y0 = y0.clamp(0, Ht - 1)
    t = tex[0]
    t00, t10, t01, t11 = t[y0, x0], t[y0, x1], t[y1, x0], t[y1, x1]
    a = t00 + (t10 - t00) * fx
    b = t01 + (t11 - t01) * fx
    return a + (b - a) * fy


def setup_reference_import():
    sys.dont_write_bytecode = True
    _stub("cv2", INTER_CUBIC=2, INTER_LINEAR=1, INTER_AREA=3)
    _stub("imageio")
    _stub("imageio.v3")
    sys.modules["imageio"].v3 = sys.modules["imageio.v3"]
    _stub("skimage")
    _stub("skimage.measure")
    _stub("plyfile", PlyData=object, PlyElement=object)
    _stub("simple_knn")
    _stub("simple_knn._C", distCUDA2=None)
    nv = _stub("nvdiffrast")
    nvt = _stub("nvdiffrast.torch", texture=texture_linear_clamp)
    nv.torch = nvt
    # map device="cuda" to CPU
    real = {}
    for fn in ["zeros", "ones", "tensor", "as_tensor", "empty", "arange", "full", "rand", "randn", "zeros_like",
               "ones_like", "empty_like", "full_like"]:
        real[fn] = getattr(torch, fn)

        def wrap(f):
            def g(*a, **k):
                if "device" in k and k["device"] is not None and "cuda" in str(k["device"]):
                    k["device"] = "cpu"
                return f(*a, **k)
            return g
        setattr(torch, fn, wrap(real[fn]))
    torch.Tensor.cuda = lambda self, *a, **k: self
    sys.path.insert(0, REF)
    pkg = types.ModuleType("scene")
    pkg.__path__ = [os.path.join(REF, "scene")]
    sys.modules["scene"] = pkg
    os.chdir(REF)  # light.py:41 loads the LUT from a cwd-relative path


def main():
    setup_reference_import()
    from utils import sh_utils
    from utils import general_utils as gu
    from utils import graphics_utils as gfx
    from scene.NVDIFFREC.light import EnvironmentLight
    from scene.gaussian_model import GaussianModel

    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(1234)
    torch.manual_seed(1234)

    # ---------------- eval_sh, deg 0..5 -----------------------------------------------
    N = 64
    fx = {}
    for deg in range(6):
        K = (deg + 1) ** 2
        sh = torch.tensor(rng.normal(0, 0.5, (N, 3, K)), dtype=torch.float32)
        d = torch.tensor(rng.normal(0, 1, (N, 3)), dtype=torch.float32)
        d = d / d.norm(dim=1, keepdim=True)
        out = sh_utils.eval_sh(deg, sh, d)
        fx[f"sh{deg}"] = sh.numpy()
        fx[f"dirs{deg}"] = d.numpy()
        fx[f"out{deg}"] = out.numpy()
    np.savez_compressed(os.path.join(OUT, "eval_sh.npz"), **fx)

    # ---------------- gauss_kernel --------------------------------------------------------
    kr = torch.tensor(rng.uniform(0, 1, (N, 1)), dtype=torch.float32)
    np.savez_compressed(os.path.join(OUT, "gauss_kernel.npz"), kr=kr.numpy(),
                        k4=sh_utils.gauss_kernel(kr, 4).numpy(), k5=sh_utils.gauss_kernel(kr, 5).numpy())

    # ---------------- shade (forward + autograd backward) --------------------------------
    lut = np.fromfile(os.path.join(REF, "scene/NVDIFFREC/irrmaps/bsdf_256_256.bin"), dtype=np.float32)
    fx = {"lut_sha256": np.frombuffer(__import__("hashlib").sha256(lut.tobytes()).digest(), np.uint8)}
    cases = [("spec_km", True, True, 4), ("spec_nokm", True, False, 4), ("diffuse", False, True, 4),
             ("spec_km_deg5", True, True, 5), ("spec_km_deg2", True, True, 2)]
    Ns = 257
    for name, specular, with_km, deg in cases:
        K = (deg + 1) ** 2
        base = torch.tensor(rng.normal(0, 0.3, (K, 3)), dtype=torch.float32)
        base[0] = 1.0
        pos = torch.tensor(rng.normal(0, 2, (Ns, 3)), dtype=torch.float32)
        campos = torch.tensor([0.3, -0.2, -4.0], dtype=torch.float32)
        view_pos = campos.repeat(Ns, 1)
        nrm = torch.tensor(rng.normal(0, 1, (Ns, 3)), dtype=torch.float32)
        nrm = nrm / nrm.norm(dim=1, keepdim=True)
        # flip towards the camera as GaussianModel.get_normal does (gaussian_model.py:115-122)
        dirpp = (pos - view_pos)
        dirpp = dirpp / dirpp.norm(dim=1, keepdim=True)
        nrm, _ = gu.flip_align_view(nrm, dirpp)
        albedo = torch.tensor(rng.uniform(0, 1, (Ns, 3)), dtype=torch.float32)
        kr_ = torch.tensor(rng.uniform(0.02, 0.98, (Ns, 1)), dtype=torch.float32)
        km_ = torch.tensor(rng.uniform(0, 1, (Ns, 1)), dtype=torch.float32)
        leaves = [t.clone().requires_grad_(True) for t in (pos, nrm, albedo, view_pos, kr_, km_, base)]
        lp, ln, la, lv, lkr, lkm, lb = leaves
        light = EnvironmentLight(base=lb, sh_degree=deg)
        light.base = lb  # keep the leaf (set_base squeezes a view; same values)
        rgb, extras = light.shade(gb_pos=lp[None, None], gb_normal=ln[None, None], albedo=la[None, None],
                                  view_pos=lv[None, None], kr=lkr[None, None],
                                  km=lkm[None, None] if with_km else None, specular=specular)
        g_rgb = torch.tensor(rng.normal(0, 1, (1, 1, Ns, 3)), dtype=torch.float32)
        g_dif = torch.tensor(rng.normal(0, 1, (1, 1, Ns, 3)), dtype=torch.float32)
        g_spe = torch.tensor(rng.normal(0, 1, (1, 1, Ns, 3)), dtype=torch.float32)
        outs = [rgb, extras["diffuse"]]
        gouts = [g_rgb, g_dif]
        if specular:
            outs.append(extras["specular"])
            gouts.append(g_spe)
        grads = torch.autograd.grad(outs, leaves, gouts, allow_unused=True)
        gnames = ["d_pos", "d_normal", "d_albedo", "d_view_pos", "d_kr", "d_km", "d_base"]
        rec = dict(pos=pos.numpy(), normal=nrm.detach().numpy(), albedo=albedo.numpy(), view_pos=view_pos.numpy(),
                   kr=kr_.numpy(), km=km_.numpy(), base=base.numpy(), with_km=np.array(with_km),
                   specular=np.array(specular), deg=np.array(deg), rgb=rgb.detach().numpy().reshape(Ns, 3),
                   diffuse=extras["diffuse"].detach().numpy().reshape(Ns, 3),
                   specular_out=extras["specular"].detach().numpy().reshape(Ns, 3),
                   g_rgb=g_rgb.numpy().reshape(Ns, 3), g_diffuse=g_dif.numpy().reshape(Ns, 3),
                   g_specular=g_spe.numpy().reshape(Ns, 3))
        for gn, gv in zip(gnames, grads):
            rec[gn] = np.zeros(0, np.float32) if gv is None else gv.numpy()
        for k, v in rec.items():
            fx[f"{name}/{k}"] = v
    np.savez_compressed(os.path.join(OUT, "shade.npz"), **fx)

    # ---------------- cov3D, normals, depth, SH->RGB, cameras -----------------------------
    P = 200
    s = torch.tensor(np.exp(rng.normal(np.log(0.05), 0.5, (P, 3))), dtype=torch.float32)
    q = torch.tensor(rng.normal(0, 1, (P, 4)), dtype=torch.float32)
    q = q / q.norm(dim=1, keepdim=True)
    mod = 1.3
    L = gu.build_scaling_rotation(mod * s, q)
    cov = gu.strip_symmetric(L @ L.transpose(1, 2))
    R = gu.build_rotation(q)
    nrm = gu.get_minimum_axis(s, R)
    xyz = torch.tensor(rng.normal(0, 1, (P, 3)) + np.array([0, 0, 5.0]), dtype=torch.float32)
    cams = {}
    cam_specs = [
        (np.eye(3), np.zeros(3), np.radians(60.0), np.radians(60.0), 256, 256),
        (None, None, 2 * np.arctan(1920 / 2800.0), 2 * np.arctan(1080 / 2800.0), 1920, 1080),
        (None, None, np.radians(50.0), np.radians(35.0), 333, 177),
    ]
    for ci, (Rm, Tv, fovx, fovy, W, H) in enumerate(cam_specs):
        if Rm is None:
            a = rng.normal(0, 0.3, 3)
            th = np.linalg.norm(a)
            k = a / th
            Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
            Rm = np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx
            Tv = rng.normal(0, 0.5, 3)
        wvt = torch.tensor(gfx.getWorld2View2(Rm, Tv)).transpose(0, 1)
        proj = gfx.getProjectionMatrix(znear=0.01, zfar=100.0, fovX=fovx, fovY=fovy).transpose(0, 1)
        full = (wvt.unsqueeze(0).bmm(proj.unsqueeze(0))).squeeze(0)
        center = wvt.inverse()[3, :3]
        cams[f"cam{ci}/R"] = Rm
        cams[f"cam{ci}/T"] = Tv
        cams[f"cam{ci}/fov"] = np.array([fovx, fovy])
        cams[f"cam{ci}/wh"] = np.array([W, H])
        cams[f"cam{ci}/viewmatrix"] = wvt.numpy()
        cams[f"cam{ci}/projmatrix"] = full.numpy()
        cams[f"cam{ci}/campos"] = center.numpy()
        ns = types.SimpleNamespace(get_xyz=xyz)
        camobj = types.SimpleNamespace(world_view_transform=wvt)
        cams[f"cam{ci}/depth"] = GaussianModel.get_depth(ns, camobj).numpy()
        dirpp = xyz - center[None]
        dirpp = dirpp / dirpp.norm(dim=1, keepdim=True)
        fl, _ = gu.flip_align_view(nrm, dirpp)
        cams[f"cam{ci}/normal_flipped"] = fl.numpy()
    # SH -> RGB with the rasterizer's convention (deg <= 3, shs [P, K, 3])
    shx = {}
    for deg in range(4):
        K = (deg + 1) ** 2
        shs = torch.tensor(rng.normal(0, 0.4, (P, 16, 3)), dtype=torch.float32)
        campos = torch.tensor(rng.normal(0, 0.5, 3), dtype=torch.float32)
        d = xyz - campos[None]
        d = d / d.norm(dim=1, keepdim=True)
        rgb = torch.clamp_min(sh_utils.eval_sh(deg, shs[:, :K, :].transpose(1, 2), d) + 0.5, 0.0)
        shx[f"shrgb{deg}/shs"] = shs.numpy()
        shx[f"shrgb{deg}/campos"] = campos.numpy()
        shx[f"shrgb{deg}/rgb"] = rgb.numpy()
    np.savez_compressed(os.path.join(OUT, "geometry.npz"), scales=s.numpy(), rotations=q.numpy(),
                        scale_modifier=np.array(mod, np.float32), cov3D=cov.numpy(), min_axis=nrm.numpy(),
                        xyz=xyz.numpy(), **cams, **shx)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
