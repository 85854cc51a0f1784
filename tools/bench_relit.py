#!/usr/bin/env python
"""Times relit_shade.relit_features alone (forward, and forward + backward of a weighted sum of
its 14 columns) at P Gaussians on one stream: HIP events over 50 back-to-back iterations each
(tools only, GPU box).  The kernels: k_relit_fwd, then k_relit_bwd and k_shade_base_reduce.

    GSR_LIB_PATH=... python tools/bench_relit.py [P]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "relightable3dgaussians-w_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402


def main():
    import relit_shade
    from test_gpu_relit import _light, _scene
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 1_500_000
    xyz, q, s, is_sky, mat, sky_sh, campos, wvt = _scene(P=P, n_sky=P // 11)
    light = _light()
    leaves = [t.clone().requires_grad_(True) for t in (xyz, q, mat["albedo"], mat["roughness"], mat["metalness"],
                                                       light.base, sky_sh)]
    x, qq, al, kr, km, base, ssh = leaves
    lt = relit_shade.EnvironmentLight(base, sh_degree=4)
    w = torch.randn(P, 14, device="cuda")

    def fwd():
        return relit_shade.relit_features(x, qq, s, is_sky, al, kr, km, lt, campos, wvt, ssh, 1, True, False)[:, :14]

    def step():
        (fwd() * w).sum().backward()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    n = 50
    with torch.no_grad():
        ev[0].record()
        for _ in range(n):
            fwd()
        ev[1].record()
    for _ in range(n):
        step()
    ev[2].record()
    torch.cuda.synchronize()
    tf = 1000 * ev[0].elapsed_time(ev[1]) / n
    ts = 1000 * ev[1].elapsed_time(ev[2]) / n
    print(f"P={P}: relit_features forward {tf:.1f} us, forward + backward {ts:.1f} us (backward ~{ts - tf:.1f} us)")


if __name__ == "__main__":
    main()
