"""Synthetic scenes and cameras for the benchmark configs (BASELINE.json configs).

Cameras follow the reference's conventions exactly:
  utils/graphics_utils.py:47-58 getWorld2View2, :60-80 getProjectionMatrix,
  scene/cameras.py:74-79 (world_view_transform = W2V^T, full_proj_transform = W2V^T @ P^T,
  camera_center = inverse(world_view_transform)[3, :3]).
The rasterizer consumes them as row-vector x row-major (auxiliary.h:58-77).

There is no dataset on the box: every config is synthetic with fixed seeds and matched
sizes (P, W, H, SH degree); data="synthetic" in every report.
"""
import math
from dataclasses import dataclass

import numpy as np
import torch

SH_C0 = 0.28209479177387814


def get_world2view2(R, t, translate=np.zeros(3), scale=1.0):
    """graphics_utils.py:47-58 (float64 math, float32 result)."""
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    cam_center = C2W[:3, 3]
    cam_center = (cam_center + translate) * scale
    C2W[:3, 3] = cam_center
    Rt = np.linalg.inv(C2W)
    return np.float32(Rt)


def get_projection_matrix(znear, zfar, fovX, fovY):
    """graphics_utils.py:60-80."""
    tanHalfFovY = math.tan((fovY / 2))
    tanHalfFovX = math.tan((fovX / 2))
    top = tanHalfFovY * znear
    bottom = -top
    right = tanHalfFovX * znear
    left = -right
    P = torch.zeros(4, 4)
    z_sign = 1.0
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = z_sign
    P[2, 2] = z_sign * zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


@dataclass
class SynthCamera:
    """Duck-types the attributes gaussian_renderer.render() reads from scene.cameras.Camera."""
    image_width: int
    image_height: int
    FoVx: float
    FoVy: float
    world_view_transform: torch.Tensor
    projection_matrix: torch.Tensor
    full_proj_transform: torch.Tensor
    camera_center: torch.Tensor
    znear: float = 0.01
    zfar: float = 100.0

    @property
    def tanfovx(self):
        return math.tan(self.FoVx * 0.5)

    @property
    def tanfovy(self):
        return math.tan(self.FoVy * 0.5)

    def to(self, device):
        return SynthCamera(self.image_width, self.image_height, self.FoVx, self.FoVy,
                           self.world_view_transform.to(device), self.projection_matrix.to(device),
                           self.full_proj_transform.to(device), self.camera_center.to(device), self.znear,
                           self.zfar)


def make_camera(W, H, FoVx, FoVy, R=None, T=None, device="cpu"):
    """scene/cameras.py:74-79 with trans = 0, scale = 1."""
    R = np.eye(3) if R is None else np.asarray(R, dtype=np.float64)
    T = np.zeros(3) if T is None else np.asarray(T, dtype=np.float64)
    wvt = torch.tensor(get_world2view2(R, T)).transpose(0, 1)
    proj = get_projection_matrix(znear=0.01, zfar=100.0, fovX=FoVx, fovY=FoVy).transpose(0, 1)
    full = (wvt.unsqueeze(0).bmm(proj.unsqueeze(0))).squeeze(0)
    center = wvt.inverse()[3, :3]
    cam = SynthCamera(int(W), int(H), float(FoVx), float(FoVy), wvt, proj, full, center)
    return cam.to(device)


def focal_camera(W, H, focal, **kw):
    return make_camera(W, H, 2 * math.atan(W / (2 * focal)), 2 * math.atan(H / (2 * focal)), **kw)


def look_at_rotation(cam_pos, target):
    """World->camera rotation R (COLMAP convention: R is stored as camera->world
    columns transposed by getWorld2View2) looking from cam_pos to target, y down."""
    f = np.asarray(target, np.float64) - np.asarray(cam_pos, np.float64)
    f /= np.linalg.norm(f)
    up = np.array([0.0, -1.0, 0.0])
    r = np.cross(up, f)
    if np.linalg.norm(r) < 1e-6:
        r = np.array([1.0, 0.0, 0.0])
    r /= np.linalg.norm(r)
    d = np.cross(f, r)
    # camera axes in world: x=r, y=d, z=f ; world2cam rotation rows are the axes
    W2C = np.stack([r, d, f], 0)
    # getWorld2View2 uses R^T as the rotation block, so R = W2C^T
    R = W2C.T
    T = -W2C @ np.asarray(cam_pos, np.float64)
    return R, T


def view_camera(cam, k):
    """View k of a multi-view run over one scene: k = 0 is `cam` itself, k > 0 a
    deterministic nearby camera (offset up to +-0.15 and looking at a point 10 units ahead,
    jittered by +-0.2), same intrinsics.  Distinct views of the same Gaussians for the
    mini-batch and data-parallel benchmarks."""
    if k == 0:
        return cam
    rng = np.random.default_rng(100 + k)
    pos = rng.uniform(-0.15, 0.15, 3)
    target = np.array([rng.uniform(-0.2, 0.2), rng.uniform(-0.2, 0.2), 10.0])
    R, T = look_at_rotation(pos, target)
    return make_camera(cam.image_width, cam.image_height, cam.FoVx, cam.FoVy, R=R, T=T,
                       device=cam.world_view_transform.device)


def rgb2sh(rgb):
    return (rgb - 0.5) / SH_C0


def synthetic_gaussians(P, W, H, tanfovx, tanfovy, sh_degree=0, seed=0, zrange=(2.0, 8.0), log_z=False,
                        scale_mode="cfg1", device="cpu", dtype=torch.float32):
    """SURVEY §8d synthetic Gaussian clouds in camera-aligned world space (camera at the origin
    looking down +z).  Returns CPU-generated tensors moved to `device`.

    cfg1: z ~ U(2,8), log-scale ~ N(ln 0.02, 0.3), opacity ~ U(0.05, 0.99).
    cfg2: z ~ logU(1,30), scale ~ exp(N(ln(0.004 z), 0.5)) -> screen radius ~10-20 px.
    """
    g = torch.Generator().manual_seed(seed)
    if log_z:
        lz = torch.empty(P).uniform_(math.log(zrange[0]), math.log(zrange[1]), generator=g)
        z = torch.exp(lz)
    else:
        z = torch.empty(P).uniform_(zrange[0], zrange[1], generator=g)
    x = torch.empty(P).uniform_(-1, 1, generator=g) * z * tanfovx
    y = torch.empty(P).uniform_(-1, 1, generator=g) * z * tanfovy
    means = torch.stack([x, y, z], 1)
    if scale_mode == "cfg1":
        scales = torch.exp(torch.empty(P, 3).normal_(math.log(0.02), 0.3, generator=g))
    else:
        scales = torch.exp(torch.empty(P, 3).normal_(0.0, 0.5, generator=g) + torch.log(0.004 * z)[:, None])
    q = torch.empty(P, 4).normal_(0, 1, generator=g)
    q = q / q.norm(dim=1, keepdim=True)
    opac = torch.empty(P, 1).uniform_(0.05, 0.99, generator=g)
    K = (sh_degree + 1) ** 2
    shs = torch.empty(P, K, 3).normal_(0, 0.2, generator=g)
    shs[:, 0, :] = rgb2sh(torch.empty(P, 3).uniform_(0, 1, generator=g))
    colors = torch.empty(P, 3).uniform_(0, 1, generator=g)
    out = dict(means3D=means, scales=scales, rotations=q, opacities=opac, shs=shs, colors=colors)
    return {k: v.to(device=device, dtype=dtype).contiguous() for k, v in out.items()}


CONFIGS = {
    # name: (P, W, H, sh_degree, camera builder, gaussian kwargs)
    "cfg1": dict(P=10_000, W=256, H=256, sh_degree=0, fov=math.radians(60.0), zrange=(2.0, 8.0), log_z=False,
                 scale_mode="cfg1"),
    "cfg2": dict(P=1_500_000, W=1920, H=1080, sh_degree=3, focal=1400.0, zrange=(1.0, 30.0), log_z=True,
                 scale_mode="cfg2"),
    "cfg5": dict(P=5_000_000, W=3840, H=2160, sh_degree=3, focal=2800.0, zrange=(1.0, 30.0), log_z=True,
                 scale_mode="cfg2"),
}


def build_config(name, device="cpu", seed=0, P=None, W=None, H=None):
    c = dict(CONFIGS[name])
    if P is not None:
        c["P"] = P
    if W is not None:
        c["W"] = W
    if H is not None:
        c["H"] = H
    if "fov" in c:
        cam = make_camera(c["W"], c["H"], c["fov"], c["fov"], device=device)
    else:
        cam = focal_camera(c["W"], c["H"], c["focal"], device=device)
    gs = synthetic_gaussians(c["P"], c["W"], c["H"], cam.tanfovx, cam.tanfovy, c["sh_degree"], seed=seed,
                             zrange=c["zrange"], log_z=c["log_z"], scale_mode=c["scale_mode"], device=device)
    return cam, gs, c


def load_ply_gaussians(path, device="cpu"):
    """A trained scene saved by GaussianModel.save_ply (scene/gaussian_model.py:296-355) as
    rasterizer inputs, with the model's activations (gaussian_model.py:54-70):
    means3D (sky Gaussians placed from their angles, :95-104), scales = exp, rotations =
    normalised, opacities = sigmoid, colors = sigmoid(albedo), plus is_sky, roughness and
    metalness (sigmoid).  Reads through the drop-in `plyfile` (plyfile.py)."""
    import plyfile
    v = plyfile.PlyData.read(path).elements[0]
    names = [p.name for p in v.properties]
    col = lambda prefix: np.stack([np.asarray(v[n], np.float32) for n in names if n.startswith(prefix)], 1)
    xyz = np.stack([np.asarray(v[k], np.float32) for k in ("x", "y", "z")], 1)
    is_sky = np.asarray(v["is_sky"]).astype(bool) if "is_sky" in names else np.zeros(len(xyz), bool)
    if is_sky.any() and "sky_radius" in names:
        ang = col("sky_angles_")[is_sky].astype(np.float64)
        th = np.clip(ang[:, 0], 0, np.pi / 2)
        ph = np.clip(ang[:, 1], -np.pi / 2, np.pi / 2)
        r = float(np.asarray(v["sky_radius"])[0])
        c = col("sky_gauss_center_")[0].astype(np.float64)
        d = np.stack([np.sin(th) * np.sin(ph), -np.cos(th), np.sin(th) * np.cos(ph)], 1)
        xyz[is_sky] = (r * d + c).astype(np.float32)
    sig = lambda a: 1.0 / (1.0 + np.exp(-a))
    rot = col("rot_")
    rot = rot / np.maximum(np.linalg.norm(rot, axis=1, keepdims=True), 1e-12)
    out = dict(means3D=xyz, scales=np.exp(col("scale_")), rotations=rot,
               opacities=sig(np.asarray(v["opacity"], np.float32))[:, None], colors=sig(col("albedo_")),
               is_sky=is_sky)
    for k in ("roughness", "metalness"):
        if k in names:
            out[k] = sig(np.asarray(v[k], np.float32))[:, None]
    return {k: torch.from_numpy(np.ascontiguousarray(a)).to(device=device,
                                                            dtype=torch.bool if a.dtype == bool else torch.float32)
            for k, a in out.items()}


def ply_config(path, W=1920, H=1080, focal=1400.0):
    """Bench inputs from a saved scene: the rasterizer's SH path at degree 0 with the albedo
    as the DC colour (so bench.py's SH3 plumbing applies unchanged), camera at the
    foreground median minus 2x the foreground extent along z, looking at it."""
    g = load_ply_gaussians(path)
    fg = g["means3D"][~g["is_sky"]] if (~g["is_sky"]).any() else g["means3D"]
    med = fg.median(dim=0).values.double().numpy()
    ext = float((fg.quantile(0.9, dim=0) - fg.quantile(0.1, dim=0)).norm())
    pos = med - np.array([0.0, 0.0, 2.0 * max(ext, 1e-3)])
    R, T = look_at_rotation(pos, med)
    cam = focal_camera(W, H, focal, R=R, T=T)
    P = g["means3D"].shape[0]
    shs = rgb2sh(g["colors"]).reshape(P, 1, 3)
    gs = dict(means3D=g["means3D"], scales=g["scales"], rotations=g["rotations"], opacities=g["opacities"],
              shs=shs.contiguous(), colors=g["colors"])
    return cam, gs, dict(P=P, W=W, H=H, sh_degree=0)
