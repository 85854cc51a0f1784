"""Drop-in `plyfile` (plyfile.py) and the PLY scene loader (gsr.scenes.load_ply_gaussians):
round trips in the reference's save_ply layout (scene/gaussian_model.py:296-355), binary
and ASCII, big-endian reads, list properties."""
import io
import math

import numpy as np
import pytest
import torch


def ref_layout(P, sky):
    """A structured array with the attributes GaussianModel.save_ply writes."""
    names = ["x", "y", "z", "albedo_0", "albedo_1", "albedo_2", "opacity", "scale_0", "scale_1", "scale_2",
             "rot_0", "rot_1", "rot_2", "rot_3", "roughness", "metalness", "is_sky"]
    if sky:
        names += ["sky_radius", "sky_gauss_center_0", "sky_gauss_center_1", "sky_gauss_center_2", "sky_angles_0",
                  "sky_angles_1"]
    rng = np.random.default_rng(1)
    arr = np.empty(P, dtype=[(n, "f4") for n in names])
    for n in names:
        arr[n] = rng.normal(size=P).astype(np.float32)
    arr["is_sky"] = (np.arange(P) % 5 == 0) if sky else 0
    if sky:
        arr["sky_radius"] = 50.0
        arr["sky_gauss_center_0"], arr["sky_gauss_center_1"], arr["sky_gauss_center_2"] = 1.0, 2.0, 3.0
    return arr


@pytest.mark.parametrize("text", [False, True])
def test_roundtrip_reference_layout(tmp_path, text):
    from plyfile import PlyData, PlyElement
    arr = ref_layout(1000, sky=True)
    p = str(tmp_path / "scene.ply")
    PlyData([PlyElement.describe(arr, "vertex")], text=text).write(p)
    d = PlyData.read(p)
    v = d.elements[0]
    assert v.name == "vertex" and v.count == 1000 and d["vertex"] is v
    assert [q.name for q in v.properties] == list(arr.dtype.names)
    for n in arr.dtype.names:
        np.testing.assert_array_equal(np.asarray(v[n]), arr[n])


def test_big_endian_and_lists():
    from plyfile import PlyData
    hdr = (b"ply\nformat binary_big_endian 1.0\ncomment test\nelement vertex 2\nproperty float x\n"
           b"property uchar flag\nelement face 1\nproperty list uchar int vertex_indices\nend_header\n")
    body = np.array([(1.5, 7), (-2.0, 9)], dtype=[("x", ">f4"), ("flag", "u1")]).tobytes()
    body += bytes([3]) + np.array([0, 1, 1], ">i4").tobytes()
    d = PlyData.read(io.BytesIO(hdr + body))
    np.testing.assert_array_equal(d["vertex"]["x"], [1.5, -2.0])
    np.testing.assert_array_equal(d["vertex"]["flag"], [7, 9])
    np.testing.assert_array_equal(d["face"]["vertex_indices"][0], [0, 1, 1])
    assert d.comments == ["test"]


def test_ascii_lists():
    from plyfile import PlyData
    txt = (b"ply\nformat ascii 1.0\nelement vertex 2\nproperty double x\nproperty int k\n"
           b"element face 2\nproperty list uchar uint idx\nend_header\n1.25 3\n-4 5\n2 0 1\n3 1 0 1\n")
    d = PlyData.read(io.BytesIO(txt))
    np.testing.assert_array_equal(d["vertex"]["x"], [1.25, -4.0])
    assert list(d["face"]["idx"][1]) == [1, 0, 1]


def test_truncated_file_is_an_error():
    from plyfile import PlyData, PlyParseError
    hdr = b"ply\nformat binary_little_endian 1.0\nelement vertex 10\nproperty float x\nend_header\n"
    with pytest.raises(PlyParseError):
        PlyData.read(io.BytesIO(hdr + b"\\0" * 12))


def test_scene_loader_activations(tmp_path):
    from plyfile import PlyData, PlyElement
    from gsr import scenes
    arr = ref_layout(500, sky=True)
    p = str(tmp_path / "s.ply")
    PlyData([PlyElement.describe(arr, "vertex")]).write(p)
    g = scenes.load_ply_gaussians(p)
    sky = arr["is_sky"].astype(bool)
    sig = lambda a: 1 / (1 + np.exp(-a.astype(np.float64)))
    np.testing.assert_allclose(g["opacities"].numpy()[:, 0], sig(arr["opacity"]), rtol=1e-6)
    np.testing.assert_allclose(g["scales"].numpy()[:, 0], np.exp(arr["scale_0"].astype(np.float64)), rtol=1e-6)
    np.testing.assert_allclose(torch.linalg.norm(g["rotations"], dim=1).numpy(), 1.0, rtol=1e-6)
    np.testing.assert_array_equal(g["means3D"].numpy()[~sky, 0], arr["x"][~sky])
    # sky Gaussians sit on the sky sphere (gaussian_model.py:95-104)
    r = np.linalg.norm(g["means3D"].numpy()[sky] - np.array([1.0, 2.0, 3.0]), axis=1)
    np.testing.assert_allclose(r, 50.0, rtol=1e-5)
    assert g["is_sky"].dtype == torch.bool and int(g["is_sky"].sum()) == int(sky.sum())
