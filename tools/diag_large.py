"""Diagnostic (GPU): the 256x192 render() fixture's means2D gradient without normal_ref, both
render paths, against the reference's (tests/golden/render_large.npz)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd"), os.path.join(ROOT, "tests")]
import test_gpu_render_golden as T  # noqa: E402
from gsr import relit  # noqa: E402

G = T.GOLDS["render_large.npz"]
case = "large_colour_debug"
want = G[f"{case}/grad_nonr/means2D"]
wfull = G[f"{case}/grad/means2D"]
res = {}
for path in ("render", "render_calls"):
    _, out, g = T._run(getattr(relit, path), case, G, skip=("normal_ref",))
    res[path] = g["means2D"].cpu().numpy()
    _, out2, g2 = T._run(getattr(relit, path), case, G)
    res[path + "_full"] = g2["means2D"].cpu().numpy()
is_sky = G["scene/is_sky"]
radii = G[f"{case}/radii"]
for k, v in res.items():
    w = wfull if k.endswith("_full") else want
    d = v - w
    print(k, "rel", np.linalg.norm(d) / np.linalg.norm(w), "norm", np.linalg.norm(v), "want", np.linalg.norm(w),
          "sky rel", np.linalg.norm(d[is_sky]) / max(np.linalg.norm(w[is_sky]), 1e-30),
          "fg rel", np.linalg.norm(d[~is_sky]) / max(np.linalg.norm(w[~is_sky]), 1e-30),
          "z max", float(np.abs(v[:, 2]).max()), "culled nz", float(np.abs(v[radii == 0]).max()))
    i = np.argsort(-np.linalg.norm(d, axis=1))[:5]
    print("  worst", i.tolist(), "mine", v[i].tolist(), "want", w[i].tolist(), "sky", is_sky[i].tolist(),
          "radii", radii[i].tolist())
print("fused vs calls (nonr)", np.linalg.norm(res["render"] - res["render_calls"]) / np.linalg.norm(res["render_calls"]))
