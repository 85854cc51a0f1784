#!/usr/bin/env python
"""Randomised sweep of the fused relightable render() step (gsr.relit.render: the fused relit
features kernels + one multi-channel composite + the image-space tail) against render()'s own
call sequence on the drop-in ops (tests/test_gpu_relit.py::_reference_render: PyTorch
per-Gaussian steps, one rasterizer call per image), on N random scenes: Gaussian count, sky
fraction, image size, camera, background (black / white / coloured), debug extras (specular
shading on, the sky SH of degree 1 as render() passes it).  Records every image's and every
leaf gradient's relative L2 error.
GPU box; test tooling.

    python tools/relit_sweep.py [N] [out.json]
"""
import json
import os
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def one(c):
    import relit_shade
    import test_gpu_relit as tr
    from gsr import relit
    from helpers import make_case
    xyz, q, s, is_sky, mat, sky_sh, _, _ = tr._scene(P=c["P"], n_sky=c["n_sky"], seed=c["seed"])
    W, H = c["W"], c["H"]
    cam, _ = make_case(P=10, W=W, H=H, camera=c["camera"])
    g = torch.Generator().manual_seed(c["seed"] + 1)
    sky_mask = (torch.rand(1, H, W, generator=g) > 0.2).float()
    view = types.SimpleNamespace(image_width=W, image_height=H, FoVx=cam.FoVx, FoVy=cam.FoVy,
                                 world_view_transform=cam.world_view_transform.cuda(),
                                 full_proj_transform=cam.full_proj_transform.cuda(),
                                 camera_center=cam.camera_center.cuda(), sky_mask=sky_mask)
    opacity = torch.rand(xyz.shape[0], 1, generator=g).cuda() * 0.9 + 0.05
    light = tr._light(seed=c["seed"] % 7)
    pipe = types.SimpleNamespace(compute_cov3D_python=False)
    bgt = torch.tensor(c["bg"], device="cuda")
    wts = {}

    def run(fn):
        leaves = [t.clone().requires_grad_(True) for t in (xyz, q, mat["albedo"], light.base, opacity)]
        pc = tr._Model(leaves[0], leaves[1], s, is_sky, dict(mat, albedo=leaves[2]), leaves[4])
        lt = relit_shade.EnvironmentLight(leaves[3], sh_degree=4)
        out = fn(pc, lt)
        loss = 0.0
        gen = torch.Generator(device="cuda").manual_seed(4)
        for k in sorted(out):
            if k in ("viewspace_points", "visibility_filter", "radii"):
                continue
            wts.setdefault(k, torch.randn(out[k].shape, device="cuda", generator=gen))
            loss = loss + (out[k] * wts[k]).sum()
        loss.backward()
        return out, [t.grad for t in leaves] + [out["viewspace_points"].grad]

    o_f, g_f = run(lambda pc, lt: relit.render(view, pc, lt, sky_sh, 1, pipe, bgt, debug=c["debug"]))
    o_r, g_r = run(lambda pc, lt: tr._reference_render(view, pc, lt, sky_sh, bgt, c["debug"]))
    img = {k: tr._rel(o_f[k], o_r[k]) for k in o_r if k not in ("viewspace_points", "visibility_filter", "radii")}
    grads = {n: tr._rel(a, b) for n, a, b in zip(["xyz", "rotation", "albedo", "base", "opacity", "means2D"], g_f, g_r)}
    return {"radii_equal": bool(torch.equal(o_f["radii"], o_r["radii"])), "image_rel_l2": img, "grad_rel_l2": grads,
            "image_max": max(img.values()), "grad_max": max(grads.values())}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "relit_sweep.json")
    rng = np.random.default_rng(606)
    rows = []
    t0 = time.time()
    for i in range(n):
        P = int(rng.integers(1500, 9000))
        bgs = [(0.0, 0.0, 0.0), (1.0, 1.0, 1.0), tuple(float(x) for x in rng.random(3))]
        c = dict(P=P, n_sky=int(P * rng.uniform(0.02, 0.2)), seed=int(rng.integers(0, 1 << 20)),
                 W=int(rng.choice([64, 96, 160, 200])), H=int(rng.choice([48, 80, 120])),
                 camera=str(rng.choice(["orbit", "identity"])), bg=bgs[int(rng.integers(0, 3))],
                 debug=bool(rng.random() < 0.5))
        r = one(c)
        rows.append({"case": c, **r})
        print(f"{i:3d} P={P:5d} sky={c['n_sky']:4d} {c['W']}x{c['H']} {c['camera']:8s} bg={tuple(round(x, 2) for x in c['bg'])} "
              f"debug={c['debug']!s:5s} radii_eq {r['radii_equal']} img {r['image_max']:.1e} grad {r['grad_max']:.1e} "
              f"({time.time() - t0:.0f} s)", flush=True)
    summary = {"cases": n, "radii_equal": sum(r["radii_equal"] for r in rows),
               "image_rel_l2_max": max(r["image_max"] for r in rows), "grad_rel_l2_max": max(r["grad_max"] for r in rows)}
    print(json.dumps(summary), flush=True)
    with open(out, "w") as f:
        json.dump({"summary": summary, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
