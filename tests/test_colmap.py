"""COLMAP model readers and the NeRF-OSR camera reader (gsr/colmap.py)
against tests/golden/colmap.npz, which the reference's own loaders produced from the
committed fixture scene (tools/gen_golden_colmap.py)."""
import os
import shutil

import numpy as np
import pytest
import torch

from gsr import colmap as cm
from gsr import scenes

GOLD = os.path.join(os.path.dirname(__file__), "golden")
SCENE = os.path.join(GOLD, "nerf_osr_scene")
SCENE_TXT = os.path.join(GOLD, "nerf_osr_scene_txt")


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(GOLD, "colmap.npz"), allow_pickle=False)


def _infos(ex, it):
    return sorted(cm.camera_infos(ex, it, "images"), key=lambda c: c.image_name)


@pytest.mark.parametrize("tag", ["bin", "txt"])
def test_cameras_match_reference(gold, tag):
    base = SCENE if tag == "bin" else SCENE_TXT
    if tag == "bin":
        ex = cm.read_extrinsics_binary(os.path.join(base, "sparse/0/images.bin"))
        it = cm.read_intrinsics_binary(os.path.join(base, "sparse/0/cameras.bin"))
    else:
        ex = cm.read_extrinsics_text(os.path.join(base, "sparse/0/images.txt"))
        it = cm.read_intrinsics_text(os.path.join(base, "sparse/0/cameras.txt"))
    infos = _infos(ex, it)
    assert [c.image_name for c in infos] == list(gold[f"{tag}_names"])
    assert [c.uid for c in infos] == list(gold[f"{tag}_uid"])
    # bit-identical to the reference's float64 arithmetic
    assert np.array_equal(np.stack([c.R for c in infos]), gold[f"{tag}_R"])
    assert np.array_equal(np.stack([c.T for c in infos]), gold[f"{tag}_T"])
    assert np.array_equal(np.array([c.FovY for c in infos]), gold[f"{tag}_fovy"])
    assert np.array_equal(np.array([c.FovX for c in infos]), gold[f"{tag}_fovx"])
    assert np.array_equal(np.array([(c.cx, c.cy) for c in infos]), gold[f"{tag}_cxcy"])
    assert np.array_equal(np.array([(c.width, c.height) for c in infos]), gold[f"{tag}_wh"])
    byname = {os.path.basename(e.name).split(".")[0]: e for e in ex.values()}
    ims = [byname[n] for n in gold[f"{tag}_names"]]
    assert [len(e.point3D_ids) for e in ims] == list(gold[f"{tag}_nxy"])
    assert np.array_equal(np.concatenate([np.asarray(e.xys, np.float64).reshape(-1, 2) for e in ims]),
                          gold[f"{tag}_xys"])
    assert np.array_equal(np.concatenate([np.asarray(e.point3D_ids, np.int64).reshape(-1) for e in ims]),
                          gold[f"{tag}_pids"])


@pytest.mark.parametrize("tag", ["bin", "txt"])
def test_points3d_match_reference(gold, tag):
    if tag == "bin":
        xyz, rgb, err = cm.read_points3D_binary(os.path.join(SCENE, "sparse/0/points3D.bin"))
    else:
        xyz, rgb, err = cm.read_points3D_text(os.path.join(SCENE_TXT, "sparse/0/points3D.txt"))
    assert np.array_equal(np.asarray(xyz, np.float64), gold[f"{tag}_xyz"])
    assert np.array_equal(np.asarray(rgb, np.float64), gold[f"{tag}_rgb"])
    assert np.array_equal(np.asarray(err, np.float64), gold[f"{tag}_err"])


def test_nerf_osr_split_and_normalisation(gold):
    train, test, norm = cm.read_nerf_osr_info(SCENE, eval=True)
    assert [c.image_name for c in train] == list(gold["train_names"])
    assert [c.image_name for c in test] == list(gold["test_names"])
    np.testing.assert_allclose(norm["translate"], gold["norm_translate"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(norm["radius"], gold["norm_radius"], rtol=1e-6)
    train2, test2, _ = cm.read_nerf_osr_info(SCENE, eval=False)
    assert [c.image_name for c in train2] == list(gold["train_names"]) and test2 == []


def test_text_fallback(tmp_path, gold):
    """readNerfOsrInfo reads the text model when the binary one is absent."""
    shutil.copytree(SCENE_TXT, tmp_path / "s")
    shutil.copytree(os.path.join(SCENE, "train"), tmp_path / "s" / "train")
    train, _, _ = cm.read_nerf_osr_info(str(tmp_path / "s"))
    assert [c.image_name for c in train] == list(gold["train_names"])


def test_text_reader_asserts_pinhole(tmp_path):
    p = tmp_path / "cameras.txt"
    p.write_text("1 SIMPLE_RADIAL 100 80 90.0 50.0 40.0 0.01\n")
    with pytest.raises(AssertionError):
        cm.read_intrinsics_text(str(p))


def test_unsupported_model_raises(tmp_path):
    cams = {1: cm.Camera(1, "OPENCV", 64, 48, np.arange(8, dtype=np.float64))}
    imgs = {1: cm.Image(1, np.array([1.0, 0, 0, 0]), np.zeros(3), 1, "a.png", np.zeros((0, 2)),
                        np.zeros(0, np.int64))}
    cm.write_intrinsics_binary(str(tmp_path / "cameras.bin"), cams)
    cm.write_extrinsics_binary(str(tmp_path / "images.bin"), imgs)
    ex = cm.read_extrinsics_binary(str(tmp_path / "images.bin"))
    it = cm.read_intrinsics_binary(str(tmp_path / "cameras.bin"))
    assert it[1].model == "OPENCV" and np.array_equal(it[1].params, np.arange(8.0))
    with pytest.raises(AssertionError):
        cm.camera_infos(ex, it, "images")


def test_binary_text_roundtrip(tmp_path):
    rng = np.random.default_rng(3)
    cams = {5: cm.Camera(5, "PINHOLE", 640, 480, rng.uniform(100, 600, 4))}
    imgs = {7: cm.Image(7, rng.normal(size=4), rng.normal(size=3), 5, "x_1.png", rng.uniform(0, 9, (3, 2)),
                        np.array([4, -1, 12]))}
    for w_c, w_i, r_c, r_i, ext in ((cm.write_intrinsics_binary, cm.write_extrinsics_binary,
                                     cm.read_intrinsics_binary, cm.read_extrinsics_binary, "bin"),
                                    (cm.write_intrinsics_text, cm.write_extrinsics_text, cm.read_intrinsics_text,
                                     cm.read_extrinsics_text, "txt")):
        w_c(str(tmp_path / f"c.{ext}"), cams)
        w_i(str(tmp_path / f"i.{ext}"), imgs)
        c2, i2 = r_c(str(tmp_path / f"c.{ext}")), r_i(str(tmp_path / f"i.{ext}"))
        assert np.array_equal(c2[5].params, cams[5].params) and (c2[5].width, c2[5].height) == (640, 480)
        assert np.array_equal(i2[7].qvec, imgs[7].qvec) and np.array_equal(i2[7].tvec, imgs[7].tvec)
        assert np.array_equal(i2[7].xys, imgs[7].xys) and list(i2[7].point3D_ids) == [4, -1, 12]
        assert i2[7].name == "x_1.png"


def test_rotmat_qvec_inverse():
    rng = np.random.default_rng(0)
    for _ in range(20):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        q = -q if q[0] < 0 else q
        np.testing.assert_allclose(cm.rotmat2qvec(cm.qvec2rotmat(q)), q, atol=1e-9)


@pytest.mark.parametrize("w,h,res,scale,want", [
    (1920, 1080, -1, 1.0, (1600, 900)), (1280, 853, -1, 1.0, (1280, 853)), (1920, 1080, 2, 1.0, (960, 540)),
    (1920, 1080, 800, 1.0, (800, 450)), (1920, 1080, 1, 2.0, (960, 540))])
def test_render_resolution(w, h, res, scale, want):
    assert cm.render_resolution(w, h, res, scale) == want


def test_render_camera_matrices():
    train, _, _ = cm.read_nerf_osr_info(SCENE)
    c = train[0]
    cam = cm.render_camera(c, resolution=1)
    ref = scenes.make_camera(c.width, c.height, c.FovX, c.FovY, R=c.R, T=c.T)
    assert (cam.image_width, cam.image_height) == (c.width, c.height)
    assert torch.equal(cam.world_view_transform, ref.world_view_transform)
    assert torch.equal(cam.full_proj_transform, ref.full_proj_transform)
    # the camera centre is the COLMAP centre -R_w2c^T t
    w2c = c.R.T
    np.testing.assert_allclose(cam.camera_center.numpy(), -w2c.T @ c.T, rtol=1e-5, atol=1e-5)
