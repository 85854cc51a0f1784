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


# ---- multi-step densification statistics and rank-consistent densify_and_prune ----------

N_STEPS, VIEWS_PER_RANK, P_STATS = 3, 2, 500


def view_stats(step, view, P=P_STATS):
    """A deterministic stand-in for one view's (dL/dmeans2D, radii)."""
    g = torch.Generator().manual_seed(1000 * step + view)
    grad = torch.randn(P, 3, generator=g)
    radii = (torch.rand(P, generator=g) * 12).int() * (torch.rand(P, generator=g) > 0.3).int()
    return grad, radii


def stats_run(rank, world):
    """N_STEPS steps; each rank renders views (step, rank*VIEWS_PER_RANK + j)."""
    from gsr import dp
    running = dict(xyz_gradient_accum=torch.zeros(P_STATS, 1), denom=torch.zeros(P_STATS, 1),
                   max_radii2D=torch.zeros(P_STATS))
    ss = dp.StepStats(P_STATS, "cpu")
    for step in range(N_STEPS):
        ss.zero()
        for r in ([rank] if world > 1 else range(2)):
            for j in range(VIEWS_PER_RANK):
                ss.add_view(*view_stats(step, r * VIEWS_PER_RANK + j))
        ss.commit(running, world=world)
    return running


def small_scene(seed=5, P_fg=400, P_sky=40):
    from gsr.train import RelitScene
    g = torch.Generator().manual_seed(seed)
    P = P_fg + P_sky
    xyz = torch.randn(P, 3, generator=g) + torch.tensor([0.0, 0.0, 5.0])
    is_sky = torch.zeros(P, dtype=torch.bool)
    is_sky[torch.randperm(P, generator=g)[:P_sky]] = True
    xyz[is_sky] = 30.0 * torch.nn.functional.normalize(xyz[is_sky], dim=1)
    scene = RelitScene(xyz, torch.randn(P, 3, generator=g) * 0.8 - 4.0, torch.randn(P, 4, generator=g),
                       torch.randn(P, 1, generator=g) * 2.0, torch.randn(P_fg, 3, generator=g),
                       torch.randn(P_fg, 1, generator=g), torch.randn(P_fg, 1, generator=g), is_sky, 2, "cpu")
    # non-trivial Adam state, identical on every rank
    scene.fp.exp_avg.copy_(torch.randn(scene.fp.n, generator=g) * 1e-3)
    scene.fp.exp_avg_sq.copy_(torch.rand(scene.fp.n, generator=g) * 1e-6)
    scene.fp.t = 7
    return scene


def densify_run(rank, world, seed=None):
    """Per-rank stats for 2 steps (different views per rank), reduced per step, then
    densify_and_prune with the shared generator.  Returns the scene."""
    from gsr import densify, dp
    scene = small_scene()
    P = scene.P
    ss = dp.StepStats(P, "cpu")
    for step in range(2):
        ss.zero()
        for r in ([rank] if world > 1 else range(2)):
            for j in range(VIEWS_PER_RANK):
                g, radii = view_stats(step, r * VIEWS_PER_RANK + j, P)
                ss.add_view(g * 0.02, radii)
        ss.commit(scene.stats, world=world)
    gen = dp.shared_generator("cpu") if seed is None else torch.Generator().manual_seed(seed)
    densify.densify_and_prune(scene, max_grad=0.02, min_opacity=0.1, extent=2.0, max_screen_size=20,
                              generator=gen)
    return scene


def run_densify(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gsr import dp
        running = stats_run(rank, world)
        scene = densify_run(rank, world)
        fp = scene.fp
        same = dp.replicas_identical([fp.flat, fp.exp_avg, fp.exp_avg_sq, scene.is_sky.to(torch.uint8),
                                      torch.tensor([scene.P, fp.t])])
        if rank == 0:
            out = {k: v.numpy() for k, v in running.items()}
            out.update(identical=np.array(same), P=np.array(scene.P), flat=fp.flat.numpy(), m=fp.exp_avg.numpy(),
                       v=fp.exp_avg_sq.numpy(), is_sky=scene.is_sky.numpy(), t=np.array(fp.t))
            np.savez(out_path, **out)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def run_identical_probe(rank, world, port, out_path):
    """replicas_identical on tensors that differ on rank 1 by one bit (-0.0 vs +0.0) and on
    tensors that agree."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gsr import dp
        a = torch.zeros(5)
        if rank == 1:
            a[2] = -0.0
        b = torch.arange(7, dtype=torch.float32)
        c = torch.ones(3 + rank)  # shapes differ
        flags = dp.replicas_identical([a, b, c])
        if rank == 0:
            np.save(out_path, np.array(flags))
        dist.barrier()
    finally:
        dist.destroy_process_group()


# ---- the training iteration's exchange: gsr.dp.finish_step, one collective per iteration ----

EX_ITERS = (14998, 14999, 15000, 15001)  # across densify_until_iter (15000)
COLLECTIVES = ("all_reduce", "all_gather", "broadcast", "reduce_scatter", "reduce", "all_to_all",
               "all_reduce_coalesced", "all_gather_into_tensor", "reduce_scatter_tensor")


def exchange_grad(it, r, n):
    return torch.randn(n, generator=torch.Generator().manual_seed(7919 * it + r))


EX_CHUNKS = 3  # the exchange's pipelined slices (forced: the test bucket is below the size floor)


def exchange_run(rank, world, chunks=EX_CHUNKS):
    """train_step's tail over EX_ITERS: each rank's flat gradient and 2 views' statistics, then
    gsr.dp.finish_step (world 1: both ranks' views in one process, the gradients summed in rank
    order) with an optimizer stand-in recording the ranges it is handed.  Returns (scene,
    per iteration (collectives finish_step reports, collectives issued as counted by wrapping
    every torch.distributed collective), per iteration the (lo, hi) ranges the optimizer got,
    per iteration the element counts the collectives carried)."""
    from gsr import dp
    counts, calls, sizes, opt = [], [], [], []
    if world > 1:
        for name in COLLECTIVES:
            orig = getattr(dist, name, None)
            if orig is not None:
                def wrap(*a, _orig=orig, _n=name, **k):
                    calls.append(_n)
                    sizes.append(int(a[0].numel()) if a and hasattr(a[0], "numel") else -1)
                    return _orig(*a, **k)
                setattr(dist, name, wrap)
    scene = small_scene()
    P, fp = scene.P, scene.fp
    for it in EX_ITERS:
        fp.zero_grad()
        ranks = [rank] if world > 1 else list(range(2))
        for r in ranks:
            fp.grad.add_(exchange_grad(it, r, fp.n))
        g2d, rad = [], []
        for r in ranks:
            for j in range(VIEWS_PER_RANK):
                g, radii = view_stats(it, r * VIEWS_PER_RANK + j, P)
                g2d.append(g * 0.02)
                rad.append(radii)
        n0 = len(calls)
        got = []
        ret = dp.finish_step(scene, g2d, rad, it, world=world, on_chunk=lambda lo, hi: got.append((lo, hi)),
                             chunks=chunks, min_chunk=1)
        counts.append((ret, len(calls) - n0))
        opt.append(got)
        sizes.append(None)  # iteration separator
    if world > 1:
        dp.sync_max_radii(scene.stats)
    per_it, cur = [], []
    for x in sizes:
        if x is None:
            per_it.append(cur)
            cur = []
        else:
            cur.append(x)
    return scene, counts, opt, per_it


def run_exchange(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        scene, counts, opt, sizes = exchange_run(rank, world)
        if rank == 0:
            out = {k: v.numpy() for k, v in scene.stats.items()}
            out.update(grad=scene.fp.grad.numpy(), counts=np.array(counts), tail=np.array(scene.fp.tail),
                       opt=np.array([r for it in opt for r in it]), opt_per_it=np.array([len(it) for it in opt]),
                       sizes=np.array([sum(it) for it in sizes]), nsizes=np.array([len(it) for it in sizes]))
            np.savez(out_path, **out)
        dist.barrier()
    finally:
        dist.destroy_process_group()


# ---- the reference loop's exchange helper (gsr.dp.ReferenceExchange) ---------------------

def refex_run(rank, world, P=300):
    """Two parameters' gradients + each rank's 2 views of statistics per iteration, over two
    iterations (statistics on, then off), through ReferenceExchange (world 1: both ranks'
    gradients summed in rank order and all views in one process)."""
    import types
    from gsr import dp
    xyz = torch.zeros(P, 3, requires_grad=True)
    alb = torch.zeros(P, 3, requires_grad=True)
    g = types.SimpleNamespace(xyz_gradient_accum=torch.zeros(P, 1), denom=torch.zeros(P, 1), max_radii2D=torch.zeros(P))
    ex = dp.ReferenceExchange([xyz, alb], P)
    issued = []
    grads = []
    for it, stats_on in ((0, True), (1, False)):
        ranks = [rank] if world > 1 else list(range(2))
        xyz.grad = sum(torch.randn(P, 3, generator=torch.Generator().manual_seed(100 * it + r)) for r in ranks)
        alb.grad = sum(torch.randn(P, 3, generator=torch.Generator().manual_seed(500 + 100 * it + r)) for r in ranks)
        g2d, rad = [], []
        for r in ranks:
            for j in range(VIEWS_PER_RANK):
                gg, radii = view_stats(it, r * VIEWS_PER_RANK + j, P)
                g2d.append(gg * 0.02)
                rad.append(radii)
        ex.add_views(g2d, rad, g.max_radii2D, stats_on)
        issued.append(ex.exchange(g, stats_on, world=world, chunks=2, min_chunk=1))
        grads.append((xyz.grad.clone(), alb.grad.clone()))
    if world > 1:
        dp.sync_max_radii({"max_radii2D": g.max_radii2D})
    return g, grads, issued


def run_refex(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g, grads, issued = refex_run(rank, world)
        if rank == 0:
            np.savez(out_path, accum=g.xyz_gradient_accum.numpy(), denom=g.denom.numpy(),
                     max_radii2D=g.max_radii2D.numpy(), xyz0=grads[0][0].numpy(), alb1=grads[1][1].numpy(),
                     issued=np.array(issued))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def refex_resize_run(rank, world, P1=200, P2=260):
    """ReferenceExchange built from the optimizer across a densify_and_prune-style resize: the
    Gaussians' Parameter replaced by a larger one (its optimizer state dropped, as
    gaussian_model.py:471-542 rebuilds it) and the statistics resized to P2 between two
    exchanges; an MLP weight that only rank 0's views reach and a sky radius ride in the same
    exchange (world 1: both ranks' gradients summed in rank order).  Returns the final
    parameters, the statistics, and whether a fixed-list exchange refused the resize."""
    import types
    from gsr import dp
    ranks = [rank] if world > 1 else list(range(2))
    gen = lambda s: torch.Generator().manual_seed(s)
    xyz = torch.nn.Parameter(torch.randn(P1, 3, generator=gen(1)))
    mlp = torch.nn.Parameter(torch.randn(8, 8, generator=gen(2)))
    sky = torch.nn.Parameter(torch.ones(1))
    opt = torch.optim.Adam([{"params": [xyz]}, {"params": [mlp]}, {"params": [sky]}], lr=0.01)
    g = types.SimpleNamespace(xyz_gradient_accum=torch.zeros(P1, 1), denom=torch.zeros(P1, 1),
                              max_radii2D=torch.zeros(P1))
    ex = dp.ReferenceExchange(optimizer=opt)
    fixed = dp.ReferenceExchange([xyz], P1)
    refused = False
    for it in range(2):
        P = xyz.shape[0]
        opt.zero_grad(set_to_none=True)
        xyz.grad = sum(torch.randn(P, 3, generator=gen(100 * it + r)) for r in ranks)
        if 0 in ranks:
            mlp.grad = torch.randn(8, 8, generator=gen(700 + it))
        sky.grad = sum(torch.randn(1, generator=gen(900 + 10 * it + r)) for r in ranks)
        g2d, rad = [], []
        for r in ranks:
            for j in range(VIEWS_PER_RANK):
                gg, radii = view_stats(it, r * VIEWS_PER_RANK + j, P)
                g2d.append(gg * 0.02)
                rad.append(radii)
        ex.add_views(g2d, rad, g.max_radii2D, True)
        ex.exchange(g, True, world=world, chunks=2, min_chunk=1)
        opt.step()
        if it == 0:  # densify: a new, larger Parameter (state rebuilt) and resized statistics
            new = torch.nn.Parameter(torch.cat([xyz.detach(), xyz.detach()[:P2 - P1] * 0.5]))
            del opt.state[xyz]
            opt.param_groups[0]["params"] = [new]
            xyz = new
            g.xyz_gradient_accum = torch.cat([g.xyz_gradient_accum, torch.zeros(P2 - P1, 1)])
            g.denom = torch.cat([g.denom, torch.zeros(P2 - P1, 1)])
            g.max_radii2D = torch.cat([g.max_radii2D, torch.zeros(P2 - P1)])
            try:
                fixed.add_views(g2d, rad, g.max_radii2D, True)
            except RuntimeError:
                refused = True
    return {"xyz": xyz.detach().numpy(), "mlp": mlp.detach().numpy(), "sky": sky.detach().numpy(),
            "accum": g.xyz_gradient_accum.numpy(), "denom": g.denom.numpy(), "refused": np.array(refused)}


def run_refex_resize(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gsr import dp
        out = refex_resize_run(rank, world)
        same = dp.replicas_identical([torch.from_numpy(out[k]) for k in ("xyz", "mlp", "sky", "accum", "denom")])
        if rank == 0:
            np.savez(out_path, same=np.array(same), **out)
        dist.barrier()
    finally:
        dist.destroy_process_group()
