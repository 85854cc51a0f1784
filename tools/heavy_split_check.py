"""Which tile-pass splits the heavy parity cases trigger: the forward's and the backward's per-band
heavy-tile counts after one forward + backward (GPU; one line per case).

  python tools/heavy_split_check.py [backward heavy bits, -1: the build's default]"""
import sys
sys.path[:0] = ["tests", "relightable3dgaussians-w_amd", "."]
import torch
import test_gpu_rasterizer as t
from gsr import _lib

bits = int(sys.argv[1]) if len(sys.argv) > 1 else -1
_lib.set_backward_heavy_bits(bits)
from diff_gaussian_rasterization import _C
for name, b in [("heavy_tiles", 8), ("dense_small", 6), ("sh3_orbit_bg", 5)]:
    case = next(c for c in t.CASES if c["name"] == name)
    if bits == -2:
        _lib.set_backward_heavy_bits(b)  # the thresholds test_backward_parity_quadrant_units uses
    cam, gs = t.make_case(P=case["P"], W=case["W"], H=case["H"], sh_degree=case.get("sh_degree", 0),
                          camera=case.get("camera", "identity"))
    gs = t.mutate(gs, case.get("mutate"))
    st = t.run_gpu(cam, gs, mode=case["mode"], sh_degree=case.get("sh_degree", 0))
    P = gs["means3D"].shape[0]
    W, H = cam.image_width, cam.image_height
    dout = torch.ones(3, H, W, device="cuda")
    _C.rasterize_gaussians_backward(st["bg"], st["means"], st["radii"], st["colors"], st["scales"], st["rots"], 1.0,
                                    st["cov3"], st["vm"], st["pm"], cam.tanfovx, cam.tanfovy, dout, st["sh"],
                                    case.get("sh_degree", 0), st["cp"], st["geom"], st["R"], st["binb"], st["img"])
    torch.cuda.synchronize()
    L = _lib.layout(P, st["R"], W, H)
    tab = t._view(st["img"], L.img_nheavy, 80, torch.int32).cpu().numpy()
    print(name, "R", st["R"], "tiles", ((W + 15) // 16) * ((H + 15) // 16), "fwd heavy", tab[40:48].tolist(),
          "bwd heavy", tab[8:16].tolist(), flush=True)
_lib.set_backward_heavy_bits(-1)
