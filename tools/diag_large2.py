"""Diagnostic (GPU): blend decisions of the 256x192 render() fixture's geometry, libgsr
against the C oracle: radii, n_contrib and colour of one drop-in call with the fixture's
relit colours replaced by a fixed random colour per Gaussian."""
import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd"), os.path.join(ROOT, "tests")]
from test_gpu_rasterizer import run_gpu, run_oracle  # noqa: E402

G = np.load(os.path.join(ROOT, "tests", "golden", "render_large.npz"))
W, H = int(G["W"]), int(G["H"])
P = G["scene/xyz"].shape[0]
q = G["scene/rotation"]
cam = types.SimpleNamespace(image_width=W, image_height=H, tanfovx=float(np.tan(G["FoVx"] / 2)),
                            tanfovy=float(np.tan(G["FoVy"] / 2)),
                            world_view_transform=torch.tensor(G["world_view_transform"]),
                            full_proj_transform=torch.tensor(G["full_proj_transform"]),
                            camera_center=torch.tensor(G["camera_center"]))
gs = {"means3D": torch.tensor(G["scene/xyz"]), "scales": torch.tensor(G["scene/scaling"]),
      "rotations": torch.tensor(q), "opacities": torch.tensor(G["scene/opacity"]),
      "colors": torch.tensor(np.random.default_rng(0).uniform(0, 1, (P, 3)).astype(np.float32))}
st = run_gpu(cam, gs, mode="colors")
ref = run_oracle(cam, gs, mode="colors")
nc_g = st["n_contrib"].reshape(H, W)
nc_r = ref["n_contrib"].reshape(H, W)
print("radii equal", np.array_equal(st["radii"].cpu().numpy(), ref["radii"]), "R", st["R"], ref["num_rendered"])
d = nc_g != nc_r
print("n_contrib mismatches", int(d.sum()), "of", W * H)
c = st["color"].cpu().numpy()
print("colour rel", np.linalg.norm(c - ref["color"]) / np.linalg.norm(ref["color"]),
      "max abs", float(np.abs(c - ref["color"]).max()))
if d.any():
    ys, xs = np.nonzero(d)
    print("first mismatches (y, x, gpu, oracle):", list(zip(ys[:10].tolist(), xs[:10].tolist(), nc_g[d][:10].tolist(),
                                                            nc_r[d][:10].tolist())))
# alpha-threshold decision flips (per (pixel, Gaussian) `alpha < 1/255` decisions that differ):
# n_contrib only sees the last contributor, but a flipped Gaussian with alpha ~ 1/255 moves the
# pixel's final transmittance by a factor (1 - alpha) ~ 0.996, while rounding moves it ~1e-6
tg, tr = st["final_T"].reshape(H, W), ref["final_T"].reshape(H, W)
rel = np.abs(tg - tr) / tr
fl = rel > 1e-3
print("final_T max rel", float(rel.max()), "flip pixels", int(fl.sum()), "ratios", (tg[fl] / tr[fl])[:20].tolist())
ys, xs = np.nonzero(fl)
print("flip pixels (y, x):", list(zip(ys[:20].tolist(), xs[:20].tolist())))
print("colour max abs outside flip pixels", float(np.abs(c - ref["color"]).reshape(3, H, W)[:, ~fl].max()))
