#!/usr/bin/env python
"""Write a synthetic scene in GaussianModel.save_ply's layout (scene/gaussian_model.py:296-355)
for exercising bench.py --ply and the loader: cfg2's cloud, raw (pre-activation) values."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd")]


def main(path, P=200_000):
    from gsr import scenes
    from plyfile import PlyData, PlyElement
    cam, gs, _ = scenes.build_config("cfg2", P=int(P))
    names = ["x", "y", "z", "albedo_0", "albedo_1", "albedo_2", "opacity", "scale_0", "scale_1", "scale_2",
             "rot_0", "rot_1", "rot_2", "rot_3", "roughness", "metalness", "is_sky"]
    arr = np.zeros(gs["means3D"].shape[0], dtype=[(n, "f4") for n in names])
    m, s, q, o, c = (gs[k].numpy() for k in ("means3D", "scales", "rotations", "opacities", "colors"))
    arr["x"], arr["y"], arr["z"] = m[:, 0], m[:, 1], m[:, 2]
    logit = lambda p: np.log(np.clip(p, 1e-6, 1 - 1e-6) / (1 - np.clip(p, 1e-6, 1 - 1e-6)))
    for i in range(3):
        arr[f"albedo_{i}"] = logit(c[:, i])
        arr[f"scale_{i}"] = np.log(s[:, i])
    for i in range(4):
        arr[f"rot_{i}"] = q[:, i]
    arr["opacity"] = logit(o[:, 0])
    PlyData([PlyElement.describe(arr, "vertex")]).write(path)
    print(path, arr.shape[0], "Gaussians")


if __name__ == "__main__":
    main(*sys.argv[1:])
