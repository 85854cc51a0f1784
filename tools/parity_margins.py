"""Measure the GPU-vs-oracle agreement of every forward parity case of
tests/test_gpu_rasterizer.py (RGB rel L2, RGB values off by > 1e-4, n_contrib mismatches,
final_T max abs diff), so the test's allowances can be set to the measured maxima.
Run on the GPU box:  python tools/parity_margins.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

import test_gpu_rasterizer as T  # noqa: E402
from helpers import make_case, rel_l2  # noqa: E402


def main():
    for case in T.CASES:
        cam, gs = make_case(P=case["P"], W=case["W"], H=case["H"], sh_degree=case.get("sh_degree", 0),
                            camera=case.get("camera", "identity"))
        gs = T.mutate(gs, case.get("mutate"))
        kw = dict(mode=case["mode"], bg=case.get("bg", (0.0, 0.0, 0.0)),
                  scale_modifier=case.get("scale_modifier", 1.0), sh_degree=case.get("sh_degree", 0))
        st = T.run_gpu(cam, gs, cov=case.get("cov", False), **kw)
        ref = T.run_oracle(cam, gs, cov3=st["cov3"].cpu().numpy() if case.get("cov") else None, **kw)
        color = st["color"].cpu().numpy()
        bad = np.abs(color - ref["color"]) > 1e-4 * max(1.0, np.abs(ref["color"]).max())
        nc = int((st["n_contrib"] != ref["n_contrib"]).sum())
        dT = float(np.abs(st["final_T"] - ref["final_T"]).max())
        print(f"{case['name']:18s} R={st['R']:8d} rgb_rel={rel_l2(color, ref['color']):.3e} "
              f"rgb_off={int(bad.sum())}/{bad.size} nc_mismatch={nc}/{st['n_contrib'].size} "
              f"finalT_maxdiff={dT:.3e} rgb_maxdiff={float(np.abs(color - ref['color']).max()):.3e}", flush=True)


if __name__ == "__main__":
    main()
