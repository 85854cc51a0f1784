"""Worker for tests/test_dp_gloo.py: one rank of the view-parallel DP step on the CPU.

Each rank renders its shard of the views with the C oracle (test infrastructure: it stands
in for libgsr.so so the collective logic runs without a GPU), accumulates per-view gradients
and densification statistics, then runs the exact gsr.dp reduction the GPU path uses, over
gloo.  Rank 0 writes the reduced tensors to an .npz for the parent to check.
"""
import math
import os

import numpy as np
import torch
import torch.distributed as dist

GRAD_KEYS = ("dL_dmeans3D", "dL_dsh", "dL_dopacity", "dL_dscales", "dL_drotations")


def scene(P=600, W=48, H=40, n_views=4, deg=1):
    from gsr import scenes
    fov = math.radians(60.0)
    cam0 = scenes.make_camera(W, H, fov, fov * H / W)
    gs = scenes.synthetic_gaussians(P, W, H, cam0.tanfovx, cam0.tanfovy, deg, seed=3)
    cams = []
    for v in range(n_views):
        a = 2 * math.pi * v / n_views
        pos = np.array([1.5 * math.sin(a), 0.3 * math.cos(a), 5.0 - 4.0 * math.cos(a) ** 2])
        R, T = scenes.look_at_rotation(pos, np.array([0.0, 0.0, 5.0]))
        cams.append(scenes.make_camera(W, H, fov, fov * H / W, R=R, T=T))
    return gs, cams, deg


def render_view(gs, cam, deg, view_id):
    from oracle import oracle as orc
    n = lambda t: t.detach().cpu().numpy().astype(np.float32)
    W, H = cam.image_width, cam.image_height
    bg = np.zeros(3, np.float32)
    args = (bg, n(gs["means3D"]), None, n(gs["opacities"]), n(gs["scales"]), n(gs["rotations"]), 1.0, None,
            n(cam.world_view_transform), n(cam.full_proj_transform), cam.tanfovx, cam.tanfovy, H, W)
    fwd = orc.forward(*args, n(gs["shs"]), deg, n(cam.camera_center))
    dout = np.random.default_rng(100 + view_id).standard_normal((3, H, W)).astype(np.float32)
    g = orc.backward(fwd, bg, n(gs["means3D"]), None, n(gs["scales"]), n(gs["rotations"]), 1.0, None,
                     n(cam.world_view_transform), n(cam.full_proj_transform), cam.tanfovx, cam.tanfovy, dout,
                     n(gs["shs"]), deg, n(cam.camera_center))
    return fwd, g


def local_step(rank, world, views=None):
    """Returns (grads list in GRAD_KEYS order, stats dict) accumulated over this rank's views."""
    from gsr import dp
    gs, cams, deg = scene()
    P = gs["means3D"].shape[0]
    views = dp.shard_views(len(cams), rank, world) if views is None else views
    grads = None
    stats = dict(xyz_gradient_accum=torch.zeros(P, 1), denom=torch.zeros(P, 1), max_radii2D=torch.zeros(P))
    for v in views:
        fwd, g = render_view(gs, cams[v], deg, v)
        gv = [torch.from_numpy(np.ascontiguousarray(g[k], np.float32)).reshape(P, -1) for k in GRAD_KEYS]
        grads = gv if grads is None else [a + b for a, b in zip(grads, gv)]
        dp.accumulate_view_stats(stats, torch.from_numpy(g["dL_dmean2D"]).float(),
                                 torch.from_numpy(fwd["radii"]).int())
    if grads is None:
        grads = [torch.zeros(P, k) for k in (3, 3 * 4, 1, 3, 4)]
    return grads, stats


def run(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gsr import dp
        grads, stats = local_step(rank, world)
        dp.all_reduce_grads(grads)
        dp.reduce_densification_stats(stats["xyz_gradient_accum"], stats["denom"], stats["max_radii2D"])
        if rank == 0:
            out = {k: t.numpy() for k, t in zip(GRAD_KEYS, grads)}
            out.update({k: v.numpy() for k, v in stats.items()})
            np.savez(out_path, **out)
        dist.barrier()
    finally:
        dist.destroy_process_group()
