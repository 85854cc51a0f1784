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


def look_at_rotation(cam_pos, target, upright=False):
    """World->camera rotation R (COLMAP convention: R is stored as camera->world
    columns transposed by getWorld2View2) looking from cam_pos to target.  upright: the
    image's down axis is world +y (COLMAP's down), so world-up content lands at the top of the
    frame (cfg2c).  The default keeps the rolled frame every earlier scene and fixture was made
    with (camera y = world -y: the image is rotated 180 degrees about the view axis)."""
    f = np.asarray(target, np.float64) - np.asarray(cam_pos, np.float64)
    f /= np.linalg.norm(f)
    up = np.array([0.0, 1.0 if upright else -1.0, 0.0])
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


def view_camera(cam, k, look=None):
    """View k of a multi-view run over one scene: k = 0 is `cam` itself, k > 0 a
    deterministic nearby camera (offset up to +-0.15 and looking at a point 10 units ahead,
    jittered by +-0.2), same intrinsics.  Distinct views of the same Gaussians for the
    mini-batch and data-parallel benchmarks.  ``look`` = dict(pos, target) of the scene's base
    camera (cfg2c): views k > 0 then stand within +-0.5 of pos and look at target +-0.5."""
    if k == 0:
        return cam
    rng = np.random.default_rng(100 + k)
    if look is not None:
        pos = np.asarray(look["pos"], np.float64) + rng.uniform(-0.5, 0.5, 3)
        target = np.asarray(look["target"], np.float64) + rng.uniform(-0.5, 0.5, 3)
        R, T = look_at_rotation(pos, target, upright=True)
        return make_camera(cam.image_width, cam.image_height, cam.FoVx, cam.FoVy, R=R, T=T,
                           device=cam.world_view_transform.device)
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


def _rotmat_to_quat(Rm):
    """Unit quaternions (r, x, y, z) whose build_rotation (general_utils.py:98-119) is ``Rm``
    [N,3,3] (Shepperd's method, float64)."""
    m = Rm
    tr = m[:, 0, 0] + m[:, 1, 1] + m[:, 2, 2]
    q = np.empty((m.shape[0], 4))
    cands = np.stack([tr, m[:, 0, 0], m[:, 1, 1], m[:, 2, 2]], 1)
    k = np.argmax(cands, 1)
    for i in range(4):
        s = k == i
        if not s.any():
            continue
        a = m[s]
        if i == 0:
            t = np.sqrt(1.0 + tr[s]) * 2
            q[s] = np.stack([0.25 * t, (a[:, 2, 1] - a[:, 1, 2]) / t, (a[:, 0, 2] - a[:, 2, 0]) / t,
                             (a[:, 1, 0] - a[:, 0, 1]) / t], 1)
        elif i == 1:
            t = np.sqrt(1.0 + a[:, 0, 0] - a[:, 1, 1] - a[:, 2, 2]) * 2
            q[s] = np.stack([(a[:, 2, 1] - a[:, 1, 2]) / t, 0.25 * t, (a[:, 0, 1] + a[:, 1, 0]) / t,
                             (a[:, 0, 2] + a[:, 2, 0]) / t], 1)
        elif i == 2:
            t = np.sqrt(1.0 + a[:, 1, 1] - a[:, 0, 0] - a[:, 2, 2]) * 2
            q[s] = np.stack([(a[:, 0, 2] - a[:, 2, 0]) / t, (a[:, 0, 1] + a[:, 1, 0]) / t, 0.25 * t,
                             (a[:, 1, 2] + a[:, 2, 1]) / t], 1)
        else:
            t = np.sqrt(1.0 + a[:, 2, 2] - a[:, 0, 0] - a[:, 1, 1]) * 2
            q[s] = np.stack([(a[:, 1, 0] - a[:, 0, 1]) / t, (a[:, 0, 2] + a[:, 2, 0]) / t,
                             (a[:, 1, 2] + a[:, 2, 1]) / t, 0.25 * t], 1)
    return q / np.linalg.norm(q, axis=1, keepdims=True)


def _frames(normals, rng):
    """Orthonormal frames [N,3,3] whose third column is ``normals`` and whose first two are a
    random in-plane pair."""
    n = normals / np.linalg.norm(normals, axis=1, keepdims=True)
    helper = np.where(np.abs(n[:, 1:2]) < 0.9, np.array([[0.0, 1.0, 0.0]]), np.array([[1.0, 0.0, 0.0]]))
    t1 = np.cross(helper, n)
    t1 /= np.linalg.norm(t1, axis=1, keepdims=True)
    t2 = np.cross(n, t1)
    a = rng.uniform(0, 2 * np.pi, n.shape[0])[:, None]
    u, v = np.cos(a) * t1 + np.sin(a) * t2, -np.sin(a) * t1 + np.cos(a) * t2
    return np.stack([u, v, n], 2)


def _trained_opacity(rng, n, lo_frac=0.15, mid_frac=0.25):
    """Opacities skewed high as after training (most surface splats near 1, a tail of
    translucent ones; the reference prunes below 0.005, gaussian_model.py:610-624)."""
    u = rng.uniform(0, 1, n)
    hi = rng.uniform(0.9, 0.995, n)
    mid = rng.uniform(0.4, 0.9, n)
    lo = rng.uniform(0.01, 0.4, n)
    return np.where(u < lo_frac, lo, np.where(u < lo_frac + mid_frac, mid, hi))


TREVI_CAMERA = dict(pos=(0.0, 0.0, 0.0), target=(0.0, -2.5, 20.0))


def trevi_like_gaussians(P, sh_degree=3, seed=0):
    """A Trevi-class clustered cloud (cfg2c; VERDICT r4 "Next" item 1): ``P`` Gaussians, 90 % on
    surface sheets and clusters of a facade scene seen from a plaza, 10 % on the reference's sky
    shell.  COLMAP axes (+y down), camera at the origin looking at (0, -2.5, 20) (TREVI_CAMERA):

      * facade (50 % of the foreground): a 32 x 9.6 m wall at z ~ 20 with column relief, density
        gradient towards the centre and the bottom (Beta-distributed x / y);
      * ground (20 %): the plaza and basin at y = 1.6, z in [-6, 20] -- its near part lies behind
        the camera or below the frame (culled);
      * sculptures (18 %): 14 anisotropic 3D clusters in front of the facade centre, Zipf-sized
        (the largest ~75k Gaussians): the dense tiles;
      * water spray (7 %): a translucent volume (opacity 0.02-0.25) in front of the centre: the
        long-list, late-saturating tiles;
      * side buildings (5 %): sheets left and right, mostly outside the frustum;
      * sky (10 % of P): sample_points_on_unit_hemisphere's band (general_utils.py:229-240;
        y ~ -0.5 U, phi in [-pi/4, pi/4]) scaled by the 0.99-quantile distance of the foreground
        from its mean and centred on the camera (get_sky_xyz_init, gaussian_model.py:211-230;
        every band point projects above 2/3 of the frame), isotropic at the shell's point spacing
        (distCUDA2's role, :249-250), opacity trained high.

    Surface splats are flat (normal axis 0.15x the in-plane scales, in-plane scales 1.2x the
    local point spacing with a log-normal spread).  Opacities follow _trained_opacity.  Returns
    the rasterizer inputs plus ``is_sky`` (CPU float32 / bool tensors)."""
    rng = np.random.default_rng(1000 + seed)
    P_sky = P // 10
    P_fg = P - P_sky
    n_fac, n_gnd, n_scu, n_spr = int(0.50 * P_fg), int(0.20 * P_fg), int(0.18 * P_fg), int(0.07 * P_fg)
    n_side = P_fg - n_fac - n_gnd - n_scu - n_spr
    xyz, nrm, s_in, s_n, opa = [], [], [], [], []

    def sheet(pts, normals, spacing, flat=0.15, op=None):
        xyz.append(pts)
        nrm.append(normals)
        si = spacing * 2.0 * np.exp(rng.normal(0.0, 0.5, (pts.shape[0], 2)))
        s_in.append(si)
        s_n.append(si.min(1) * flat)
        opa.append(_trained_opacity(rng, pts.shape[0]) if op is None else op)

    # facade: x in [-16, 16], y in [-8, 1.6] (bottom denser), column relief in z
    x = 16.0 * (2 * rng.beta(1.6, 1.6, n_fac) - 1)
    y = 1.6 - 9.6 * rng.beta(1.2, 2.0, n_fac)
    z = 20.0 - 0.6 * np.sin(x * 1.3) ** 8 + rng.normal(0, 0.08, n_fac)
    sheet(np.stack([x, y, z], 1), np.tile([0.0, 0.0, -1.0], (n_fac, 1)) + rng.normal(0, 0.15, (n_fac, 3)),
          math.sqrt(32 * 9.6 / n_fac))
    # ground: the plaza / basin
    x = rng.uniform(-18, 18, n_gnd)
    z = -6.0 + 26.0 * rng.beta(1.0, 1.6, n_gnd)
    y = 1.6 + rng.normal(0, 0.02, n_gnd)
    sheet(np.stack([x, y, z], 1), np.tile([0.0, -1.0, 0.0], (n_gnd, 1)) + rng.normal(0, 0.1, (n_gnd, 3)),
          math.sqrt(36 * 26 / n_gnd))
    # sculptures: Zipf-sized anisotropic clusters
    nc = 14
    w = 1.0 / np.arange(1, nc + 1) ** 1.1
    cnt = np.floor(w / w.sum() * n_scu).astype(np.int64)
    cnt[0] += n_scu - cnt.sum()
    for c in range(nc):
        ctr = np.array([rng.uniform(-6, 6), rng.uniform(-3.5, 1.0), rng.uniform(16.5, 19.5)])
        sig = rng.uniform(0.25, 1.0, 3) * np.array([1.0, 1.4, 0.6])
        pts = ctr + rng.normal(0, 1, (cnt[c], 3)) * sig
        vol = 4.0 / 3.0 * math.pi * float(np.prod(2 * sig))
        sheet(pts, rng.normal(0, 1, (cnt[c], 3)), (vol / cnt[c]) ** (1.0 / 3.0), flat=0.3)
    # water spray: translucent, small, in front of the centre
    pts = np.stack([rng.normal(0, 1.2, n_spr), rng.uniform(-1.2, 1.6, n_spr), rng.normal(16.0, 0.9, n_spr)], 1)
    sheet(pts, rng.normal(0, 1, (n_spr, 3)), 0.035, flat=0.6, op=rng.uniform(0.02, 0.25, n_spr))
    # side buildings
    side = np.where(rng.uniform(0, 1, n_side) < 0.5, -1.0, 1.0)
    x = side * rng.uniform(16, 30, n_side)
    pts = np.stack([x, rng.uniform(-10, 1.6, n_side), rng.uniform(6, 40, n_side)], 1)
    sheet(pts, np.stack([-side, np.zeros(n_side), np.zeros(n_side)], 1) + rng.normal(0, 0.2, (n_side, 3)),
          math.sqrt(14 * 11.6 * 34 * 2 / 14 / n_side))
    fg = np.concatenate(xyz)
    # the reference's sky band around the camera centre (the only camera)
    dist = np.linalg.norm(fg - fg.mean(0), axis=1)
    sky_distance = float(np.quantile(dist, 0.99))
    yb = -0.5 * rng.uniform(0, 1, P_sky)
    th = np.arccos(yb)
    ph = 0.5 * np.pi * rng.uniform(0, 1, P_sky) - np.pi / 4
    band = np.stack([np.sin(ph) * np.sin(th), yb, np.sin(th) * np.cos(ph)], 1)
    sky = band * sky_distance + np.asarray(TREVI_CAMERA["pos"])
    area = sky_distance ** 2 * (0.5 * np.pi) * 0.5
    sp = math.sqrt(area / P_sky)
    sky_s = sp * 1.5 * np.exp(rng.normal(0.0, 0.3, P_sky))
    all_xyz = np.concatenate([fg, sky])
    frames = _frames(np.concatenate(nrm), rng)
    scales = np.concatenate([np.concatenate([np.concatenate(s_in), np.concatenate(s_n)[:, None]], 1),
                             np.repeat(sky_s[:, None], 3, 1)])
    q = np.concatenate([_rotmat_to_quat(frames), np.tile([1.0, 0.0, 0.0, 0.0], (P_sky, 1))])
    opac = np.concatenate([np.concatenate(opa), rng.uniform(0.85, 0.99, P_sky)])[:, None]
    K = (sh_degree + 1) ** 2
    shs = rng.normal(0, 0.2, (P, K, 3))
    shs[:, 0, :] = rgb2sh(rng.uniform(0, 1, (P, 3)))
    colors = rng.uniform(0, 1, (P, 3))
    is_sky = np.zeros(P, bool)
    is_sky[P_fg:] = True
    out = dict(means3D=all_xyz, scales=scales, rotations=q, opacities=opac, shs=shs, colors=colors)
    out = {k: torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32)) for k, v in out.items()}
    out["is_sky"] = torch.from_numpy(is_sky)
    return out


CONFIGS = {
    # name: (P, W, H, sh_degree, camera builder, gaussian kwargs)
    "cfg1": dict(P=10_000, W=256, H=256, sh_degree=0, fov=math.radians(60.0), zrange=(2.0, 8.0), log_z=False,
                 scale_mode="cfg1"),
    "cfg2": dict(P=1_500_000, W=1920, H=1080, sh_degree=3, focal=1400.0, zrange=(1.0, 30.0), log_z=True,
                 scale_mode="cfg2"),
    # cfg2's size on a Trevi-class clustered cloud (trevi_like_gaussians)
    "cfg2c": dict(P=1_500_000, W=1920, H=1080, sh_degree=3, focal=1400.0, clustered=True, look=TREVI_CAMERA),
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
    if c.get("clustered"):
        R, T = look_at_rotation(TREVI_CAMERA["pos"], TREVI_CAMERA["target"], upright=True)
        cam = focal_camera(c["W"], c["H"], c["focal"], R=R, T=T, device=device)
        gs = trevi_like_gaussians(c["P"], c["sh_degree"], seed=seed)
        gs = {k: v.to(device) for k, v in gs.items()}
        return cam, gs, c
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
