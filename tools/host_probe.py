import os, sys, time
sys.path[:0] = ["/root/repo", "/root/repo/relightable3dgaussians-w_amd"]
import torch
from diff_gaussian_rasterization import _C
from gsr import scenes
dev = torch.device("cuda", 0)
cam, gs, c = scenes.build_config("cfg2", device="cpu", seed=0)
g = {k: v.to(dev) for k, v in gs.items()}
W, H, deg = cam.image_width, cam.image_height, c["sh_degree"]
e = torch.empty(0, device=dev); bg = torch.zeros(3, device=dev)
vm, pm, cp = cam.world_view_transform.to(dev), cam.full_proj_transform.to(dev), cam.camera_center.to(dev)
dout = torch.randn(3, H, W, device=dev)
tf = tb = 0.0
def pair(meas=False):
    global tf, tb
    t0 = time.perf_counter()
    R, color, radii, geom, binb, img = _C.rasterize_gaussians(bg, g["means3D"], e, g["opacities"], g["scales"], g["rotations"], 1.0, e, vm, pm, cam.tanfovx, cam.tanfovy, H, W, g["shs"], deg, cp, False)
    t1 = time.perf_counter()
    out = _C.rasterize_gaussians_backward(bg, g["means3D"], radii, e, g["scales"], g["rotations"], 1.0, e, vm, pm, cam.tanfovx, cam.tanfovy, dout, g["shs"], deg, cp, geom, R, binb, img)
    t2 = time.perf_counter()
    if meas: tf += t1 - t0; tb += t2 - t1
    return out
for _ in range(20): pair()
torch.cuda.synchronize()
for N in (20, 100, 20, 100):
    tf = tb = 0.0
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(N): pair(True)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / N * 1e3
    print(f"N={N} wall per pair {wall:.4f} ms; host in forward call {tf/N*1e3:.4f} ms, in backward call {tb/N*1e3:.4f} ms")
N = 200
# GPU-only per pair with events around a batch
s, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(N): pair()
en.record(); torch.cuda.synchronize()
print(f"event span per pair {s.elapsed_time(en)/N:.4f} ms")

# how much GPU work is still queued when the forward call returns (an event recorded right
# after it returns completes when that work is done)
lag = []
for _ in range(30):
    R, color, radii, geom, binb, img = _C.rasterize_gaussians(bg, g["means3D"], e, g["opacities"], g["scales"], g["rotations"], 1.0, e, vm, pm, cam.tanfovx, cam.tanfovy, H, W, g["shs"], deg, cp, False)
    t_ret = time.perf_counter()
    ev = torch.cuda.Event()
    ev.record()
    ev.synchronize()
    lag.append((time.perf_counter() - t_ret) * 1e3)
    _C.rasterize_gaussians_backward(bg, g["means3D"], radii, e, g["scales"], g["rotations"], 1.0, e, vm, pm, cam.tanfovx, cam.tanfovy, dout, g["shs"], deg, cp, geom, R, binb, img)
lag.sort()
print(f"GPU work queued at the forward's return: median {lag[len(lag)//2]:.4f} ms (min {lag[0]:.4f}, max {lag[-1]:.4f})")
