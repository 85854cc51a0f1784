"""COLMAP model I/O and the NeRF-OSR camera reader, so the benchmarks can
render trained scenes from their real cameras.

Readers mirror the reference's `scene/colmap_loader.py` (same function names, namedtuple
fields and error behaviour):
  read_intrinsics_binary / _text   colmap_loader.py:203-230 / :144-166 (the text reader
                                   asserts PINHOLE, as the reference does)
  read_extrinsics_binary / _text   colmap_loader.py:168-201 / :232-259
  read_points3D_binary / _text     colmap_loader.py:113-142 / :83-111
  qvec2rotmat / rotmat2qvec        colmap_loader.py:43-66
The scene reader follows `readNerfOsrInfo` + `readColmapCameras` (scene/dataset_readers.py:
76-126, 153-210): binary model first, text on failure; cameras sorted by image name;
train/test split by the file names under <path>/train/rgb and <path>/test/rgb;
`getNerfppNorm` (:53-74).  Images and masks are not decoded: the benchmark needs geometry
only, so each camera's size comes from its intrinsics (`loadCam` then applies the
reference's resolution rule, utils/camera_utils.py:20-40).

Binary files are parsed with `struct.unpack_from` over one buffer (the reference reads
byte by byte through a file object); the writers exist for tests and tools.
"""
from __future__ import annotations

import collections
import math
import os
import struct

import numpy as np

CameraModel = collections.namedtuple("CameraModel", ["model_id", "model_name", "num_params"])
Camera = collections.namedtuple("Camera", ["id", "model", "width", "height", "params"])
BaseImage = collections.namedtuple("Image", ["id", "qvec", "tvec", "camera_id", "name", "xys", "point3D_ids"])

CAMERA_MODELS = (
    CameraModel(0, "SIMPLE_PINHOLE", 3), CameraModel(1, "PINHOLE", 4), CameraModel(2, "SIMPLE_RADIAL", 4),
    CameraModel(3, "RADIAL", 5), CameraModel(4, "OPENCV", 8), CameraModel(5, "OPENCV_FISHEYE", 8),
    CameraModel(6, "FULL_OPENCV", 12), CameraModel(7, "FOV", 5), CameraModel(8, "SIMPLE_RADIAL_FISHEYE", 4),
    CameraModel(9, "RADIAL_FISHEYE", 5), CameraModel(10, "THIN_PRISM_FISHEYE", 12),
)
CAMERA_MODEL_IDS = {m.model_id: m for m in CAMERA_MODELS}
CAMERA_MODEL_NAMES = {m.model_name: m for m in CAMERA_MODELS}


def qvec2rotmat(qvec):
    w, x, y, z = (float(v) for v in qvec)
    return np.array([
        [1 - 2 * y ** 2 - 2 * z ** 2, 2 * x * y - 2 * w * z, 2 * z * x + 2 * w * y],
        [2 * x * y + 2 * w * z, 1 - 2 * x ** 2 - 2 * z ** 2, 2 * y * z - 2 * w * x],
        [2 * z * x - 2 * w * y, 2 * y * z + 2 * w * x, 1 - 2 * x ** 2 - 2 * y ** 2]])


def rotmat2qvec(R):
    """Largest-eigenvector quaternion (w, x, y, z) with w >= 0."""
    Rxx, Ryx, Rzx, Rxy, Ryy, Rzy, Rxz, Ryz, Rzz = np.asarray(R, np.float64).flat
    K = np.array([
        [Rxx - Ryy - Rzz, 0, 0, 0],
        [Ryx + Rxy, Ryy - Rxx - Rzz, 0, 0],
        [Rzx + Rxz, Rzy + Ryz, Rzz - Rxx - Ryy, 0],
        [Ryz - Rzy, Rzx - Rxz, Rxy - Ryx, Rxx + Ryy + Rzz]]) / 3.0
    vals, vecs = np.linalg.eigh(K)
    q = vecs[[3, 0, 1, 2], np.argmax(vals)]
    return -q if q[0] < 0 else q


class Image(BaseImage):
    def qvec2rotmat(self):
        return qvec2rotmat(self.qvec)


# ---- binary ---------------------------------------------------------------------------
class _Buf:
    def __init__(self, path):
        with open(path, "rb") as f:
            self.b = f.read()
        self.o = 0

    def take(self, fmt):
        v = struct.unpack_from("<" + fmt, self.b, self.o)
        self.o += struct.calcsize("<" + fmt)
        return v

    def cstr(self):
        e = self.b.index(b"\x00", self.o)
        s = self.b[self.o:e].decode("utf-8")
        self.o = e + 1
        return s


def read_intrinsics_binary(path):
    r = _Buf(path)
    n = r.take("Q")[0]
    cams = {}
    for _ in range(n):
        cid, mid, w, h = r.take("iiQQ")
        m = CAMERA_MODEL_IDS[mid]
        cams[cid] = Camera(id=cid, model=m.model_name, width=w, height=h, params=np.array(r.take("d" * m.num_params)))
    assert len(cams) == n
    return cams


def read_extrinsics_binary(path):
    r = _Buf(path)
    n = r.take("Q")[0]
    imgs = {}
    for _ in range(n):
        p = r.take("idddddddi")
        name = r.cstr()
        n2 = r.take("Q")[0]
        a = np.frombuffer(r.b, dtype=np.dtype([("x", "<f8"), ("y", "<f8"), ("id", "<i8")]), count=n2, offset=r.o)
        r.o += 24 * n2
        imgs[p[0]] = Image(id=p[0], qvec=np.array(p[1:5]), tvec=np.array(p[5:8]), camera_id=p[8], name=name,
                           xys=np.column_stack([a["x"], a["y"]]) if n2 else np.zeros((0, 2)),
                           point3D_ids=a["id"].astype(np.int64))
    return imgs


def read_points3D_binary(path):
    r = _Buf(path)
    n = r.take("Q")[0]
    xyzs, rgbs, errors = np.empty((n, 3)), np.empty((n, 3)), np.empty((n, 1))
    for i in range(n):
        p = r.take("QdddBBBd")
        xyzs[i], rgbs[i], errors[i] = p[1:4], p[4:7], p[7]
        tl = r.take("Q")[0]
        r.o += 8 * tl  # track: (image_id i32, point2D_idx i32) pairs, unused
    return xyzs, rgbs, errors


# ---- text -----------------------------------------------------------------------------
def _lines(path):
    with open(path, "r") as f:
        for line in f:
            line = line.strip()
            if line and line[0] != "#":
                yield line


def read_intrinsics_text(path):
    cams = {}
    for line in _lines(path):
        e = line.split()
        cid, model = int(e[0]), e[1]
        assert model == "PINHOLE", "While the loader support other types, the rest of the code assumes PINHOLE"
        cams[cid] = Camera(id=cid, model=model, width=int(e[2]), height=int(e[3]),
                           params=np.array(tuple(map(float, e[4:]))))
    return cams


def read_extrinsics_text(path):
    imgs = {}
    with open(path, "r") as f:
        while True:
            line = f.readline()
            if not line:
                break
            line = line.strip()
            if not line or line[0] == "#":
                continue
            e = line.split()
            iid = int(e[0])
            pts = f.readline().split()
            imgs[iid] = Image(id=iid, qvec=np.array(tuple(map(float, e[1:5]))),
                              tvec=np.array(tuple(map(float, e[5:8]))), camera_id=int(e[8]), name=e[9],
                              xys=np.column_stack([tuple(map(float, pts[0::3])), tuple(map(float, pts[1::3]))]),
                              point3D_ids=np.array(tuple(map(int, pts[2::3]))))
    return imgs


def read_points3D_text(path):
    rows = [line.split() for line in _lines(path)]
    if not rows:
        return None, None, None  # the reference returns None for an empty file
    xyz = np.array([tuple(map(float, r[1:4])) for r in rows])
    rgb = np.array([tuple(map(int, r[4:7])) for r in rows])
    err = np.array([float(r[7]) for r in rows])
    return xyz, rgb, err


# ---- writers (tests / tools) ----------------------------------------------------------
def write_intrinsics_binary(path, cams):
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", len(cams)))
        for c in cams.values():
            m = CAMERA_MODEL_NAMES[c.model]
            f.write(struct.pack("<iiQQ", c.id, m.model_id, c.width, c.height))
            f.write(struct.pack("<" + "d" * m.num_params, *[float(v) for v in c.params]))


def write_extrinsics_binary(path, imgs):
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", len(imgs)))
        for im in imgs.values():
            f.write(struct.pack("<idddddddi", im.id, *[float(v) for v in im.qvec], *[float(v) for v in im.tvec],
                                im.camera_id))
            f.write(im.name.encode("utf-8") + b"\x00")
            f.write(struct.pack("<Q", len(im.point3D_ids)))
            for (x, y), pid in zip(im.xys, im.point3D_ids):
                f.write(struct.pack("<ddq", float(x), float(y), int(pid)))


def write_points3D_binary(path, xyz, rgb, err, tracks=None):
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", len(xyz)))
        for i in range(len(xyz)):
            f.write(struct.pack("<QdddBBBd", i + 1, *map(float, xyz[i]), *map(int, rgb[i]), float(err[i])))
            t = [] if tracks is None else tracks[i]
            f.write(struct.pack("<Q", len(t)))
            for a, b in t:
                f.write(struct.pack("<ii", a, b))


def write_intrinsics_text(path, cams):
    with open(path, "w") as f:
        f.write("# Camera list with one line of data per camera:\n")
        for c in cams.values():
            f.write(f"{c.id} {c.model} {c.width} {c.height} " + " ".join(repr(float(v)) for v in c.params) + "\n")


def write_extrinsics_text(path, imgs):
    with open(path, "w") as f:
        f.write("# Image list with two lines of data per image:\n")
        for im in imgs.values():
            f.write(f"{im.id} " + " ".join(repr(float(v)) for v in (*im.qvec, *im.tvec)) +
                    f" {im.camera_id} {im.name}\n")
            f.write(" ".join(f"{float(x)!r} {float(y)!r} {int(p)}" for (x, y), p in zip(im.xys, im.point3D_ids))
                    + "\n")


def write_points3D_text(path, xyz, rgb, err):
    with open(path, "w") as f:
        f.write("# 3D point list with one line of data per point:\n")
        for i in range(len(xyz)):
            f.write(f"{i + 1} " + " ".join(repr(float(v)) for v in xyz[i]) + " " +
                    " ".join(str(int(v)) for v in rgb[i]) + f" {float(err[i])!r}\n")


# ---- NeRF-OSR scene cameras -------------------------------------------------------------
def focal2fov(focal, pixels):
    return 2 * math.atan(pixels / (2 * focal))


def fov2focal(fov, pixels):
    return pixels / (2 * math.tan(fov / 2))


CameraInfo = collections.namedtuple("CameraInfo", ["uid", "R", "T", "FovY", "FovX", "cx", "cy", "image_path",
                                                   "image_name", "width", "height"])


def read_model_cameras(sparse_dir):
    """(extrinsics, intrinsics): binary first, text on any failure (dataset_readers.py:154-163)."""
    try:
        return (read_extrinsics_binary(os.path.join(sparse_dir, "images.bin")),
                read_intrinsics_binary(os.path.join(sparse_dir, "cameras.bin")))
    except Exception:
        return (read_extrinsics_text(os.path.join(sparse_dir, "images.txt")),
                read_intrinsics_text(os.path.join(sparse_dir, "cameras.txt")))


def camera_infos(extrinsics, intrinsics, images_folder):
    """readColmapCameras (dataset_readers.py:76-126) without decoding images.  R is the
    transposed world-to-camera rotation, T the COLMAP translation.  SIMPLE_PINHOLE takes
    its principal point from params[1:3] (the reference leaves cx/cy unset there)."""
    out = []
    for key in extrinsics:
        ex = extrinsics[key]
        it = intrinsics[ex.camera_id]
        if it.model == "SIMPLE_PINHOLE":
            f, cx, cy = it.params[0], it.params[1], it.params[2]
            fovy, fovx = focal2fov(f, it.height), focal2fov(f, it.width)
        elif it.model == "PINHOLE":
            fx, fy, cx, cy = it.params[0], it.params[1], it.params[-2], it.params[-1]
            fovy, fovx = focal2fov(fy, it.height), focal2fov(fx, it.width)
        else:
            raise AssertionError("Colmap camera model not handled: only undistorted datasets (PINHOLE or "
                                 "SIMPLE_PINHOLE cameras) supported!")
        path = os.path.join(images_folder, os.path.basename(ex.name))
        out.append(CameraInfo(uid=it.id, R=np.transpose(qvec2rotmat(ex.qvec)), T=np.array(ex.tvec), FovY=fovy,
                              FovX=fovx, cx=cx, cy=cy, image_path=path,
                              image_name=os.path.basename(path).split(".")[0], width=it.width, height=it.height))
    return out


def nerfpp_norm(infos):
    """getNerfppNorm (dataset_readers.py:53-74)."""
    from .scenes import get_world2view2
    centers = [np.linalg.inv(get_world2view2(c.R, c.T).astype(np.float64))[:3, 3:4] for c in infos]
    centers = np.hstack(centers)
    center = centers.mean(axis=1, keepdims=True)
    diagonal = np.max(np.linalg.norm(centers - center, axis=0, keepdims=True))
    return {"translate": -center.flatten(), "radius": diagonal * 1.1}


def _names(d):
    return {n.split(".")[0] for n in os.listdir(d)} if os.path.isdir(d) else None


def read_nerf_osr_info(path, images=None, eval=False):
    """readNerfOsrInfo (dataset_readers.py:153-210), cameras only: returns (train, test,
    nerf_normalization).  Without a <path>/train/rgb folder every camera is a training
    camera (the reference requires the folder)."""
    ex, it = read_model_cameras(os.path.join(path, "sparse/0"))
    infos = sorted(camera_infos(ex, it, os.path.join(path, "images" if images is None else images)),
                   key=lambda c: c.image_name)
    tr = _names(os.path.join(path, "train", "rgb"))
    train = [c for c in infos if tr is None or c.image_name in tr]
    test = []
    if eval:
        te = _names(os.path.join(path, "test", "rgb")) or set()
        test = [c for c in infos if c.image_name in te]
    return train, test, nerfpp_norm(train) if train else None


def render_resolution(width, height, resolution=-1, resolution_scale=1.0):
    """loadCam's image size rule (utils/camera_utils.py:20-40)."""
    if resolution in (1, 2, 4, 8):
        return round(width / (resolution_scale * resolution)), round(height / (resolution_scale * resolution))
    if resolution == -1:
        down = width / 1600 if width > 1600 else 1
    else:
        down = width / resolution
    s = float(down) * float(resolution_scale)
    return int(width / s), int(height / s)


def render_camera(info, resolution=-1, resolution_scale=1.0, device="cpu"):
    """A rasterizer camera (scene/cameras.py:74-79) for one CameraInfo."""
    from .scenes import make_camera
    W, H = render_resolution(info.width, info.height, resolution, resolution_scale)
    return make_camera(W, H, info.FovX, info.FovY, R=info.R, T=info.T, device=device)
