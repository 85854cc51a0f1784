"""Golden vectors for the COLMAP / NeRF-OSR camera reader (gsr/colmap.py).

1. Writes a small synthetic NeRF-OSR-layout scene with this repo's writers:
     tests/golden/nerf_osr_scene/sparse/0/{cameras,images,points3D}.bin
     tests/golden/nerf_osr_scene/{train,test}/rgb/<name>.jpg   (empty marker files)
     tests/golden/nerf_osr_scene_txt/sparse/0/{cameras,images,points3D}.txt
2. Reads them back with the REFERENCE's own loaders (scene/colmap_loader.py, imported
   read-only from /root/reference with the stub recipe of tools/gen_golden.py) and stores
   what the reference's readColmapCameras / readNerfOsrInfo derive from them (R, T, FoVs,
   principal point, sorted names, train/test split, getNerfppNorm) in
   tests/golden/colmap.npz.

Run in the build container:  python tools/gen_golden_colmap.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "relightable3dgaussians-w_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
GOLD = os.path.join(ROOT, "tests", "golden")


def make_scene():
    from gsr import colmap as cm
    rng = np.random.default_rng(77)
    scene = os.path.join(GOLD, "nerf_osr_scene")
    txt = os.path.join(GOLD, "nerf_osr_scene_txt")
    for d in (os.path.join(scene, "sparse", "0"), os.path.join(txt, "sparse", "0"),
              os.path.join(scene, "train", "rgb"), os.path.join(scene, "test", "rgb")):
        os.makedirs(d, exist_ok=True)
    cams = {
        1: cm.Camera(1, "PINHOLE", 1920, 1080, np.array([1400.5, 1398.25, 961.0, 538.5])),
        2: cm.Camera(2, "PINHOLE", 1280, 853, np.array([1000.0, 1001.5, 640.25, 426.0])),
    }
    imgs = {}
    order = rng.permutation(9)  # ids not in name order
    for k in range(9):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        q = -q if q[0] < 0 else q
        n2 = int(rng.integers(0, 4))
        imgs[k + 1] = cm.Image(id=k + 1, qvec=q, tvec=rng.normal(0, 2, 3), camera_id=1 + (k % 2),
                               name=f"img_{int(order[k]):03d}.jpg", xys=rng.uniform(0, 500, (n2, 2)),
                               point3D_ids=rng.integers(-1, 50, n2))
    xyz = rng.normal(0, 3, (40, 3))
    rgb = rng.integers(0, 256, (40, 3))
    err = rng.uniform(0, 2, 40)
    tracks = [[(int(rng.integers(1, 10)), int(rng.integers(0, 100))) for _ in range(int(rng.integers(0, 4)))]
              for _ in range(40)]
    cm.write_intrinsics_binary(os.path.join(scene, "sparse/0/cameras.bin"), cams)
    cm.write_extrinsics_binary(os.path.join(scene, "sparse/0/images.bin"), imgs)
    cm.write_points3D_binary(os.path.join(scene, "sparse/0/points3D.bin"), xyz, rgb, err, tracks)
    cm.write_intrinsics_text(os.path.join(txt, "sparse/0/cameras.txt"), cams)
    cm.write_extrinsics_text(os.path.join(txt, "sparse/0/images.txt"), imgs)
    cm.write_points3D_text(os.path.join(txt, "sparse/0/points3D.txt"), xyz, rgb, err)
    names = sorted(im.name.split(".")[0] for im in imgs.values())
    for i, n in enumerate(names):
        split = "test" if i % 4 == 0 else "train"
        open(os.path.join(scene, split, "rgb", n + ".jpg"), "wb").close()
    return scene, txt


def main():
    scene, txt = make_scene()
    from gen_golden import setup_reference_import
    setup_reference_import()
    from scene import colmap_loader as rl
    from scene.dataset_readers import getNerfppNorm
    from utils.graphics_utils import focal2fov

    out = {}
    for tag, ex_r, in_r, base in (("bin", rl.read_extrinsics_binary, rl.read_intrinsics_binary, scene),
                                  ("txt", rl.read_extrinsics_text, rl.read_intrinsics_text, txt)):
        ext = "bin" if tag == "bin" else "txt"
        ex = ex_r(os.path.join(base, "sparse/0", f"images.{ext}"))
        it = in_r(os.path.join(base, "sparse/0", f"cameras.{ext}"))
        rows = []
        for key in ex:  # readColmapCameras (dataset_readers.py:76-126), image decoding left out
            e, c = ex[key], it[ex[key].camera_id]
            R = np.transpose(rl.qvec2rotmat(e.qvec))
            rows.append((os.path.basename(e.name).split(".")[0], c.id, R, np.array(e.tvec),
                         focal2fov(c.params[1], c.height), focal2fov(c.params[0], c.width), c.params[-2],
                         c.params[-1], c.width, c.height, e.xys, e.point3D_ids))
        rows.sort(key=lambda r: r[0])
        out[f"{tag}_names"] = np.array([r[0] for r in rows])
        out[f"{tag}_uid"] = np.array([r[1] for r in rows])
        out[f"{tag}_R"] = np.stack([r[2] for r in rows])
        out[f"{tag}_T"] = np.stack([r[3] for r in rows])
        out[f"{tag}_fovy"] = np.array([r[4] for r in rows])
        out[f"{tag}_fovx"] = np.array([r[5] for r in rows])
        out[f"{tag}_cxcy"] = np.array([(r[6], r[7]) for r in rows])
        out[f"{tag}_wh"] = np.array([(r[8], r[9]) for r in rows])
        out[f"{tag}_nxy"] = np.array([len(r[10]) for r in rows])
        out[f"{tag}_xys"] = np.concatenate([np.asarray(r[10], np.float64).reshape(-1, 2) for r in rows])
        out[f"{tag}_pids"] = np.concatenate([np.asarray(r[11], np.int64).reshape(-1) for r in rows])
        pts = (rl.read_points3D_binary(os.path.join(base, "sparse/0/points3D.bin")) if tag == "bin" else
               rl.read_points3D_text(os.path.join(base, "sparse/0/points3D.txt")))
        out[f"{tag}_xyz"], out[f"{tag}_rgb"], out[f"{tag}_err"] = (np.asarray(a, np.float64) for a in pts)
    train = set(n.split(".")[0] for n in os.listdir(os.path.join(scene, "train/rgb")))
    test = set(n.split(".")[0] for n in os.listdir(os.path.join(scene, "test/rgb")))
    out["train_names"] = np.array([n for n in out["bin_names"] if n in train])
    out["test_names"] = np.array([n for n in out["bin_names"] if n in test])

    class _C:  # getNerfppNorm reads .R and .T only
        def __init__(self, R, T):
            self.R, self.T = R, T

    sel = [i for i, n in enumerate(out["bin_names"]) if n in train]
    norm = getNerfppNorm([_C(out["bin_R"][i], out["bin_T"][i]) for i in sel])
    out["norm_translate"] = np.asarray(norm["translate"], np.float64)
    out["norm_radius"] = np.float64(norm["radius"])
    np.savez_compressed(os.path.join(GOLD, "colmap.npz"), **out)
    print("wrote", os.path.join(GOLD, "colmap.npz"), sorted(out))


if __name__ == "__main__":
    main()
