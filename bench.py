#!/usr/bin/env python
"""bench.py -- MPix/s fwd+bwd of the MI355X rasterizer on BASELINE.json's headline config.

Workload (BASELINE.json configs[1], SURVEY §8d cfg 2): 1.5M synthetic Gaussians, SH degree 3,
1920x1080.  A step is 4 views per GPU at every N (cfg4's per-GPU mini-batch), each one
rasterizer forward + backward through the drop-in diff_gaussian_rasterization._C (libgsr.so,
hand-written gfx950 HIP) -- the reference's call pair, inputs resident in HBM -- the views
alternating over 3 HIP streams by default (--streams 1: one after another on one stream; the
layout is in config.views_per_step / config.streams).  With --gpus N > 1 (one process per GPU, launched by
torch.distributed.run) every rank holds the same replicated scene and renders its own 4
distinct views per step, and the per-Gaussian gradients of the step are summed over ranks with
one RCCL all-reduce (weak scaling: view-parallel data parallelism).  The per-rank
work is the same at every N, so the driver's value(N) / (N value(1)) compares like with like.

Prints ONE JSON line (rank 0).  value = whole-job MPix/s = N * V * W * H / step time (max over
ranks).  Beside it: `single_call` = SURVEY §8d's definition (median of 50 call pairs, HIP
events), `minibatch_4view` = 4 distinct cameras on 3 HIP streams (throughput).  roofline: the
dominant kernel by HIP-event time inside the timed region -- the tile passes are VALU-issue
bound, so for them `bound` is "valu" (PMC instruction count / live launch time against the
spec issue rate) with the HBM view (SURVEY §8d algorithmic bytes, PMC traffic) under
`roofline.hbm`.  cpu_baseline: the naive PyTorch-CPU rasterizer (oracle/torch_raster.py) on
this host's cores (count stated), cfg2 sampled + extrapolated and cfg1's forward in full.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "relightable3dgaussians-w_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
METRIC = "MPix/s fwd+bwd, 1.5M Gaussians @1080p; train iters/s at 1/2/4/8 GPUs"


def algorithmic_bytes(stage, P, Pv, R, T, Npix, M):
    """SURVEY §8d per-stage compulsory HBM bytes (each array touched once)."""
    S = 12 * M if M else 12
    F = 4 * TRAIN_NCH  # the relit composite's float channels per Gaussian (gsr.relit.RELIT_CHANNELS)
    return {
        "preprocess": P * 12 + Pv * (32 + S) + P * 8 + Pv * 67,
        "render_fwd": T * 8 + R * 40 + Npix * 20,
        "render_bwd": T * 8 + R * 40 + Npix * 20 + Pv * 44,
        # the multi-channel composite: §8d's terms with nch channels in place of 3 colours
        "render_fwd_mc": T * 8 + R * (28 + F) + Npix * (F + 8),
        "render_bwd_mc": T * 8 + R * (28 + F) + Npix * (8 + F) + Pv * (44 + F),
        # this design's compulsory bytes: reads radii, the 9-float accumulator line,
        # means, scales, rotations, SH; writes every output row of every Gaussian (the reference's
        # zero-filled buffers: dmean2D, dcolor, dopacity, dmean3D, dcov3D, dscale, drot, dsh)
        "preprocess_bwd": P * (4 + 36 + 12 + 12 + 16 + 12 * M) + P * (12 + 12 + 4 + 12 + 24 + 12 + 16 + 12 * M),
    }.get(stage)


STAGE_KERNEL = {"preprocess": "k_preprocess", "render_fwd": "k_render_fwd", "render_bwd": "k_render_bwd",
                "preprocess_bwd": "k_preprocess_bwd", "render_fwd_mc": "k_render_fwd_mc",
                "render_bwd_mc": "k_render_bwd_mc", "shade_fwd": "k_shade_fwd", "shade_bwd": "k_shade_bwd"}
# the relit legs' kernel-level stages (render_fwd / render_bwd also hold the order launch)
RELIT_STAGES = ("preprocess", "depth_sort", "st_emit", "render_fwd_mc", "render_bwd_mc", "preprocess_bwd",
                "shade_fwd", "shade_bwd")


# spec VALU issue rate: a wave64 VALU instruction issues over 2 cycles on a SIMD-32, 2.4 GHz
# (MI355X_MICROARCH.md "Execution model"); 1024 SIMDs -> 1228.8 G wave-instructions/s
VALU_CLOCK_GHZ = 2.4
SETTLE_STEPS = 16  # untimed steps right before the timed region, at least (W warmup + settle)
VALU_CYCLES_PER_INST = 2


def _pmc_record(stage, workload):
    """The newest committed rocprofv3 record (profiles/r*_hbm_traffic.json, tools/profile_summary.py)
    of the stage's kernel whose profiled bench line ran the same workload; ({}, None) if none.
    Newest = the latest `created` stamp; records written before the stamp existed rank below
    every stamped one, among themselves by tag."""
    import glob
    recs = [(json.load(open(f)), f) for f in glob.glob(os.path.join(ROOT, "profiles", "r*_hbm_traffic.json"))]
    for d, f in sorted(recs, key=lambda r: (r[0].get("created", ""), os.path.basename(r[1])), reverse=True):
        b = d.get("bench_under_profiler") or {}
        if (b.get("config") or {}).get("workload", "").split(",")[0] != workload.split(",")[0]:
            continue
        ks = d.get("kernels", {})
        want = STAGE_KERNEL.get(stage, "")
        name = want if want in ks else next((k for k in ks if k.startswith(want + "<")), None)  # template args
        return (ks.get(name, {}) if name else {}), os.path.relpath(f, ROOT)
    return {}, None


def pmc_kernel(stage, workload):
    return _pmc_record(stage, workload)


def pmc_traffic(stage, workload):
    """HBM bytes per launch of the stage's kernel from the newest committed rocprofv3 PMC pass
    of this same workload (profiles/<tag>_hbm_traffic.json, written by tools/profile_summary.py
    from separate --pmc FETCH_SIZE / WRITE_SIZE runs of this bench command, corrected as
    MI355X_MICROARCH.md prescribes).  None when no such profile exists."""
    k, src = _pmc_record(stage, workload)
    return k.get("traffic_bytes"), src


def unique_bytes(stage, P, Pv, R, T, Npix, M):
    """Compulsory HBM bytes of the tile passes if every array were read once: each visible
    Gaussian's 48-B record and its super-tile entries (~1.5 per Gaussian at 8 B; the tile
    passes filter each tile's list from them, no R-sized point list exists), the image state,
    the gradient lines.  SURVEY §8d's figure counts one 40-B record read per instance (R x 40)
    instead; the records are re-read from L2 across the tiles a Gaussian touches."""
    return {"render_fwd": T * 8 + Pv * (48 + 12) + Npix * 20,
            "render_bwd": T * 8 + Pv * (48 + 12) + Npix * 20 + Pv * 44}.get(stage)


STAGE_VIEWS = 24  # views (one at a time, one stream) behind stage_ms


def stage_breakdown(view, n):
    """Per-stage HIP-event times over ``n`` views run one at a time on one stream:
    {stage: (total ms, launches)}."""
    from gsr import _lib
    _lib.profile_read(reset=True)
    _lib.profile_stages(None)
    _lib.profile_enable(True)
    for _ in range(n):
        view()
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    return _lib.profile_read(reset=True)


def single_call_median(view, W, H, n=50, warm=10):
    """SURVEY §8d's definition: W*H / (t_fwd + t_bwd) of ONE call, the median of ``n`` calls
    after ``warm`` warm-up, HIP events on the stream the calls run on."""
    for _ in range(warm):
        view()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in evs:
        a.record()
        view()
        b.record()
    torch.cuda.synchronize()
    t_ms = sorted(a.elapsed_time(b) for a, b in evs)
    med = t_ms[len(t_ms) // 2]
    return {"median_ms": round(med, 4), "p10_ms": round(t_ms[n // 10], 4), "p90_ms": round(t_ms[(9 * n) // 10], 4),
            "calls": len(t_ms), "value": round(W * H / (med * 1e-3) / 1e6, 3), "unit": "MPix/s",
            "what": f"one rasterizer forward + backward call pair, median of {n} (HIP events, {warm} warm-up)"}


def _null_over_peak(view, keys=("frac", "unique_frac")):
    """An HBM view whose bytes / time exceed the HBM peak was served partly from L2 / Infinity
    Cache: its fraction is no HBM fraction, so it is nulled (the cfg5-relit leg's HBM
    sub-view printed 2.08), the raw achieved GB/s kept."""
    for k in keys:
        v = view.get(k)
        if v is not None and v > 1.0:
            view[k] = None
            view[k + "_null_reason"] = ("bytes / launch time exceed the HBM peak: served partly from L2 / Infinity "
                                        "Cache, so no HBM fraction")
    return view


def tile_roofline(dom, P, Pv, R, T, W, H, M, workload, dev):
    """The roofline object of the dominant stage ``dom`` = (stage, avg launch ms)."""
    dom_bytes = algorithmic_bytes(dom[0], P, Pv, R, T, W * H, M)
    traffic, traffic_src = pmc_traffic(dom[0], workload)
    if dom_bytes is None or dom[1] <= 0:  # a stage without a §8d byte count (or not timed)
        return {"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None,
                "traffic": None if traffic is None else int(traffic), "kernel": dom[0],
                "avg_launch_ms": round(dom[1], 4), "frac_null_reason": f"no SURVEY §8d byte count for stage {dom[0]}"}
    achieved_gbs = dom_bytes / (dom[1] * 1e-3) / 1e9
    hbm = {"achieved": round(achieved_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved_gbs / HBM_PEAK_GBS, 5), "bytes": "algorithmic (SURVEY §8d per-stage figure x "
                                                                   "this launch's measured P, P_v, R)",
           "algorithmic_bytes_per_launch": int(dom_bytes),
           "traffic": None if traffic is None else int(traffic), "traffic_source": traffic_src}
    ub = unique_bytes(dom[0], P, Pv, R, T, W * H, M)
    if ub is not None:
        hbm["unique_bytes_per_launch"] = int(ub)
        hbm["unique_frac"] = round(ub / (dom[1] * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
    _null_over_peak(hbm)
    kinfo, ksrc = pmc_kernel(dom[0], workload)
    if kinfo.get("valu_insts") and dom[0].startswith("render"):
        # The tile passes are bound by VALU issue (the PMC counters show their HBM traffic at
        # ~0.3x the algorithmic bytes): instruction throughput against the spec issue rate,
        # 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction (MI355X_MICROARCH.md).
        n_simd = 4 * torch.cuda.get_device_properties(dev).multi_processor_count
        peak = n_simd * VALU_CLOCK_GHZ / VALU_CYCLES_PER_INST
        ach = kinfo["valu_insts"] / (dom[1] * 1e-3) / 1e9
        roofline = {"bound": "valu", "achieved": round(ach, 1), "peak": round(peak, 1), "unit": "Gwave-inst/s",
                    "frac": round(ach / peak, 4), "traffic": hbm["traffic"], "kernel": dom[0],
                    "avg_launch_ms": round(dom[1], 4), "valu_insts_per_launch": int(kinfo["valu_insts"]),
                    "valu_source": ksrc,
                    "peak_basis": f"{n_simd} SIMDs x {VALU_CLOCK_GHZ} GHz / {VALU_CYCLES_PER_INST} cycles per "
                                  "wave64 VALU instruction (spec issue rate)",
                    "hbm": hbm}
        if kinfo.get("salu_insts"):
            # the scalar instructions the same waves issue (mask logic, walk bookkeeping,
            # branches): a co-bound, DESIGN.md §3 (an added SALU op per evaluation costs more
            # than an added VALU op)
            roofline["salu_insts_per_launch"] = int(kinfo["salu_insts"])
            roofline["salu_per_valu"] = round(kinfo["salu_insts"] / kinfo["valu_insts"], 3)
    elif dom[0].startswith("render"):
        # a tile pass with no committed instruction count for this workload: its bound is VALU
        # issue, and the HBM fraction of its algorithmic bytes is not a roofline
        # (the R x 40 record reads are served from LDS/L2), so no fraction is claimed
        roofline = {"bound": "valu", "achieved": None, "peak": None, "unit": "Gwave-inst/s", "frac": None,
                    "traffic": hbm["traffic"], "kernel": dom[0], "avg_launch_ms": round(dom[1], 4),
                    "frac_null_reason": f"no committed rocprofv3 SQ_INSTS_VALU pass of workload '{workload}' "
                                        "(profiles/r*_hbm_traffic.json)", "hbm": hbm}
    else:
        roofline = {"bound": "hbm", "achieved": hbm["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": hbm["frac"], "traffic": hbm["traffic"], "kernel": dom[0],
                    "avg_launch_ms": round(dom[1], 4), "hbm": hbm}
    if roofline["bound"] == "hbm" and roofline["frac"] is not None and roofline["frac"] > 1.0:
        # more algorithmic bytes per second than HBM delivers: part of them came from a cache,
        # so the figure is no HBM fraction
        roofline.update(frac=None, frac_null_reason="algorithmic bytes / launch time exceed the HBM peak (served "
                                                    "from L2 / Infinity Cache)")
    return roofline


def cpu_baseline(cam, gs_cpu, deg, dout_cpu, ntiles=64, seed=2, cfg1=True):
    """The north star's naive PyTorch-CPU rasterizer (oracle/torch_raster.py, checked against
    the C oracle by tests/test_torch_raster_cpu.py) on this host's cores.  cfg2: the full
    preprocess and binning of all P Gaussians, render forward + backward on `ntiles` random
    tiles (seed 2) extrapolated by tile count, and the full preprocess backward (autograd).
    cfg1 (10k Gaussians, 256x256, SH0): the whole forward, timed in full."""
    from gsr import scenes
    from oracle import torch_raster as tr
    threads = tr.host_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        W, H = cam.image_width, cam.image_height
        bg = torch.zeros(3)
        t0 = time.perf_counter()
        leaves = [gs_cpu["means3D"].clone().requires_grad_(True), gs_cpu["scales"].clone().requires_grad_(True),
                  gs_cpu["rotations"].clone().requires_grad_(True), gs_cpu["shs"].clone().requires_grad_(True)]
        pre = tr.preprocess(leaves[0], leaves[1], leaves[2], gs_cpu["opacities"], leaves[3], deg,
                            cam.world_view_transform.cpu(), cam.full_proj_transform.cpu(), cam.camera_center.cpu(), W,
                            H, cam.tanfovx, cam.tanfovy)
        with torch.no_grad():
            pl, ranges = tr.binning(pre, W, H)
        t1 = time.perf_counter()
        T = ranges.shape[0]
        tiles = tr.sample_tiles(T, ntiles, seed)
        xy, con, rgb = pre["xy"], pre["conic"].detach(), pre["rgb"].detach()
        with torch.no_grad():
            color, fT, nc, _ = tr.render_fwd(tiles, ranges, pl, xy, con, pre["opacity"], rgb, bg, W, H)
            t2 = time.perf_counter()
            rb = tr.render_bwd(gs_cpu["means3D"].shape[0], tiles, ranges, pl, xy, con, pre["opacity"], rgb, bg, fT, nc,
                               tr.from_image(dout_cpu, tiles, W, H), W, H)
        t3 = time.perf_counter()
        tr.preprocess_bwd(pre, leaves, rb["dL_dmean2D"], rb["dL_dconic"], rb["dL_dcolors"])
        t4 = time.perf_counter()
        est = (t1 - t0) + (t3 - t1) * T / len(tiles) + (t4 - t3)
        out = dict(value=W * H / est / 1e6, unit="MPix/s", cores=threads, kind="port",
                   sample=(f"cfg2 ({gs_cpu['means3D'].shape[0]} Gaussians, {W}x{H}, SH{deg}): naive PyTorch-CPU "
                           f"rasterizer (oracle/torch_raster.py) on {threads} threads; full preprocess + binning "
                           f"(R={pl.numel()}, {t1 - t0:.2f} s) and preprocess backward ({t4 - t3:.2f} s), render "
                           f"fwd+bwd on {len(tiles)}/{T} random tiles (seed {seed}, {t3 - t1:.2f} s) extrapolated "
                           f"by tile count; estimated {est:.1f} s per fwd+bwd"),
                   seconds_per_fwd_bwd_estimated=round(est, 3))
        if cfg1:
            c1cam, c1gs, _ = scenes.build_config("cfg1", device="cpu", seed=0)
            tc0 = time.perf_counter()
            tr.rasterize(c1gs["means3D"], c1gs["scales"], c1gs["rotations"], c1gs["opacities"], c1gs["shs"], 0,
                         c1cam.world_view_transform, c1cam.full_proj_transform, c1cam.camera_center, 256, 256,
                         c1cam.tanfovx, c1cam.tanfovy, torch.zeros(3))
            tc = time.perf_counter() - tc0
            out["cfg1_forward"] = {"seconds": round(tc, 4), "mpix_per_s": round(256 * 256 / tc / 1e6, 4),
                                   "what": "cfg1 (10k Gaussians, 256x256, SH0) whole forward, timed in full"}
        return out
    finally:
        torch.set_num_threads(prev)


class _RelitModel:
    """The GaussianModel properties render() reads (scene/gaussian_model.py:74-180), as
    plain tensors of a synthetic scene."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


class _WeightedSum(torch.autograd.Function):
    """The relit legs' training-style loss: sum over render()'s images of <image, weights>
    (fixed random weights), as one dot product per image instead of a product image, a sum
    and a scalar add per image; the backward writes weights x dL into the composite's gradient
    rows when render() reserved them (gsr.relit.slab_take), so its channel split copies
    nothing.  Same value and gradient as sum((out[k] * w[k]).sum())."""

    @staticmethod
    def forward(ctx, weights, *imgs):
        ctx.weights, ctx.imgs = weights, imgs
        return torch.stack([torch.dot(i.reshape(-1), w.reshape(-1)) for i, w in zip(imgs, weights)]).sum()

    @staticmethod
    def backward(ctx, g):
        from gsr import relit
        grads = []
        for i, w in zip(ctx.imgs, ctx.weights):
            dst = relit.slab_take(i) if i.is_contiguous() else None
            if dst is not None and dst.shape == w.shape:
                torch.mul(w, g, out=dst)
                grads.append(dst)
            else:
                grads.append(w * g)
        ctx.imgs = None
        return (None, *grads)


def bench_relight(args, dev):
    """--config cfg3 / cfg5-relit: relight_leg as the JSON line."""
    print(json.dumps(relight_leg(args, dev, args.config == "cfg5-relit", args.steps, args.warmup,
                                 with_calls=not args.fused_only)), flush=True)


def relight_leg(args, dev, stress, steps, warmup, with_calls=True, P_fg=None):
    """cfg3: the relightable render() step (gaussian_renderer/__init__.py:69-280,
    debug=False) and a training-style loss backward through all of its images (render,
    diffuse, specular, depth, normal, alpha, normal_ref).  value = views/s of the fused path
    (gsr.relit.render: relit features + one multi-channel composite); render()'s own call
    sequence on the drop-in ops (gsr.relit.render_calls: PyTorch per-Gaussian steps + six
    rasterizer calls), with and without the geometry cache, is reported beside it
    (with_calls, cfg3 only).  stress: cfg5 -- 5M Gaussians at 3840x2160."""
    import types

    import diff_gaussian_rasterization as dgr
    import relit_shade
    from gsr import relit, scenes, shrot
    P_fg = P_fg or args.P or (4_545_455 if stress else 1_000_000)
    P = P_fg + P_fg // 10  # + 10 % sky Gaussians
    cam, gs, c = scenes.build_config("cfg5" if stress else "cfg2", device="cpu", seed=0, P=P)
    W, H = cam.image_width, cam.image_height
    gen = torch.Generator().manual_seed(7)
    is_sky = torch.zeros(P, dtype=torch.bool)
    is_sky[P_fg:] = True
    leaves = {"xyz": gs["means3D"], "rotation": gs["rotations"], "opacity": gs["opacities"],
              "albedo": torch.rand(P_fg, 3, generator=gen), "roughness": torch.rand(P_fg, 1, generator=gen) * 0.9 + 0.05,
              "metalness": torch.rand(P_fg, 1, generator=gen)}
    leaves = {k: v.to(dev) for k, v in leaves.items()}
    scaling = gs["scales"].to(dev)
    base = torch.randn(25, 3, generator=gen) * 0.3
    base[0] = 1.0
    # the reference's relight sequence (relit_novel_view.py:131-152): the environment SH
    # rotated about y by 30 angles over [0, 6.28], one view per angle, fix_sky=True with a
    # zero sky SH
    bases = [b.to(dev) for b in shrot.rotated_sequence(base)]
    sky_sh = torch.zeros(1, 4, 3, device=dev)
    view = types.SimpleNamespace(image_width=W, image_height=H, FoVx=cam.FoVx, FoVy=cam.FoVy,
                                 world_view_transform=cam.world_view_transform.to(dev),
                                 full_proj_transform=cam.full_proj_transform.to(dev),
                                 camera_center=cam.camera_center.to(dev), sky_mask=torch.ones(1, H, W, device=dev))
    pipe = types.SimpleNamespace(compute_cov3D_python=False)
    bg = torch.zeros(3, device=dev)
    names = ("render", "diffuse_color", "specular_color", "depth", "normal", "alpha", "normal_ref")
    dweights = {k: torch.randn(3, H, W, generator=gen).to(dev) for k in names}
    dweights_t = tuple(dweights[k] for k in names)

    is_sky_dev = is_sky.to(dev)[:, None]  # one device tensor: render()'s foreground index stays cached
    # consecutive views (the relight sequence of relit_novel_view.py renders one view per env
    # rotation) are independent: they alternate over HIP streams, each view's backward on its
    # forward's stream
    nsr = max(1, 2 if args.streams is None else args.streams)
    main_s = torch.cuda.current_stream(dev)
    rstreams = [main_s] if nsr == 1 else [torch.cuda.Stream(dev) for _ in range(nsr)]
    counter = [0]

    def step(fn):
        k = counter[0]
        s = rstreams[k % len(rstreams)]
        counter[0] += 1
        s.wait_stream(main_s)
        with torch.cuda.stream(s):
            t = {k_: v.detach().requires_grad_(True) for k_, v in leaves.items()}
            light = relit_shade.EnvironmentLight(bases[k % len(bases)].detach().clone().requires_grad_(True),
                                                 sh_degree=4)
            pc = _RelitModel(get_xyz=t["xyz"], get_rotation=t["rotation"], get_scaling=scaling,
                             get_opacity=t["opacity"], get_is_sky=is_sky_dev, get_albedo=t["albedo"],
                             get_roughness=t["roughness"], get_metalness=t["metalness"])
            out = fn(view, pc, light, sky_sh, 1, pipe, bg, debug=False, fix_sky=True)
            loss = _WeightedSum.apply(dweights_t, *[out[k] for k in names])
            loss.backward()

    def timed(fn):
        for _ in range(warmup):
            step(fn)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step(fn)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / steps

    ms = timed(relit.render)
    # the dominant kernel's live launch time (HIP events on its stream, views one at a time on
    # one stream after the timed region) and the measured R, P_v of one more view
    from gsr import _lib
    saved = rstreams[:]
    rstreams[:] = [main_s]
    _lib.profile_read(reset=True)
    _lib.profile_stages(list(RELIT_STAGES))
    _lib.profile_enable(True)
    for _ in range(max(1, args.event_steps)):
        step(relit.render)
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    live = _lib.profile_read(reset=True)
    _lib.profile_stages(None)
    dgr.record_channels_calls(True)
    step(relit.render)
    torch.cuda.synchronize()
    dgr.record_channels_calls(False)
    rstreams[:] = saved
    R, Pv = int(dgr.last_channels_call["num_rendered"]), int(dgr.last_channels_call["visible"])
    stage_ms = {k: v[0] / v[1] for k, v in live.items() if v[1] > 0}
    dom = max(((k, v) for k, v in stage_ms.items() if k in RELIT_STAGES), key=lambda kv: kv[1],
              default=("render_bwd_mc", 0.0))
    workload = f"{'cfg5 (relit stress)' if stress else 'cfg3'}: {P_fg} foreground + {P - P_fg} sky Gaussians"
    roof = tile_roofline(dom, P, Pv, R, ((W + 15) // 16) * ((H + 15) // 16), W, H, 0, workload, dev)
    roof["stage_ms"] = {k: round(v, 4) for k, v in stage_ms.items()}
    res = {True: float("nan"), False: float("nan")}
    if with_calls and not stress:
        for cached in (True, False):
            dgr.geometry_cache(cached)
            res[cached] = timed(relit.render_calls)
        dgr.geometry_cache(True)
    return {
        "metric": "relit render() views/s (render()'s images + training loss backward)", "value": round(1e3 / ms, 3),
        "unit": "views/s", "n_gpus": 1, "steps": steps, "warmup": warmup, "ms_per_step": round(ms, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"{'cfg5 (relit stress)' if stress else 'cfg3'}: {P_fg} foreground + {P - P_fg} sky "
                               f"Gaussians, {W}x{H}, env SH deg 4 rotated about y over the reference's 30 relight "
                               "angles (one per view), fix_sky=True, debug=False", "gaussians": P,
                   "width": W, "height": H},
        "mpix_per_s": round(W * H / (ms * 1e-3) / 1e6, 3),
        "roofline": roof, "measured": {"num_rendered": R, "visible": Pv},
        "implementation": f"gsr.relit.render: fused relit features + one 14-channel composite; views on {nsr} "
                          "HIP streams",
        "loss": "hand-fused dot-product loss (_WeightedSum: sum over render()'s images of <image, fixed random "
                "weights>, its gradient written into render()'s composite gradient rows; since round 5, d35eeb0) -- "
                "not the reference's L1 + D-SSIM + sky-BRDF + normal composition, which the train leg runs",
        "render_calls": None if res[True] != res[True] else {
            "cached_ms": round(res[True], 4), "uncached_ms": round(res[False], 4),
            "fused_speedup_vs_cached": round(res[True] / ms, 3)}}


TRAIN_VIEWS_PER_RANK = 4
TRAIN_ITERATION = 15001  # past reg_normal_from_iter (15000): the normal-consistency term is on
TRAIN_NCH = 14  # channels of the fused render()'s composite (gsr.relit.RELIT_CHANNELS)
TRAIN_DOM_KERNEL = "k_render_bwd_mc"


def train_algorithmic_bytes(P, P_fg, Pv, R, T, Npix, V, n_params, nch=TRAIN_NCH):
    """Compulsory HBM bytes of one cfg4 iteration (each array touched once), by kernel family.
    The rasterizer terms are SURVEY §8d's B_fwd / B_bwd with the composite's nch float channels
    in place of the 3 colours (a record read per instance: id 4 + xy 8 + conic/opacity 16 +
    4 nch feature bytes; nch planes out, nch gradient planes in); the shade is §8d's B_shade;
    the rest counts the arrays the iteration's other kernels must read and write once."""
    F = 4 * nch
    per_view = {
        "relit_features": P * (12 + 16 + 12 + F) + P_fg * 20,  # xyz, rotation, scale, materials -> features
        "shade": P_fg * (80 + 136),  # §8d B_shade forward + backward
        "preprocess": P * 12 + Pv * 44 + P * 8 + Pv * 67,
        "binning": P * 8 + P * 4 + Pv * 16 + R * 12 + R * 24 + R * 8 + T * 16,  # scan, duplicate, sort, ranges
        "render_fwd_mc": T * 8 + R * (28 + F) + Npix * (F + 8),
        "render_bwd_mc": T * 8 + R * (28 + F) + Npix * (8 + F) + Pv * (44 + F),
        "preprocess_bwd": P * 108 + P * 4 + Pv * 88 + P * 4 + Pv * 143,
        "relit_features_bwd": P * (F + 12 + 16 + 12) + P * 40 + P_fg * 20,  # dL/dfeatures + inputs -> grads
        # losses, SSIM and the normal epilogue: the nch planes, target, masks and the SSIM maps
        # forward (28 planes); the maps, planes and their gradients backward (42 planes)
        "image_space": Npix * 4 * (28 + 42),
    }
    per_iter = {"activations": n_params * 16,  # raw params -> activated, activated grads -> raw grads
                "adam": n_params * 28,  # param, grad, two moments read; param, two moments written
                "densify_stats": V * P * 16}
    return V * sum(per_view.values()) + sum(per_iter.values()), per_view, per_iter


def _pmc_train_record():
    """The newest committed rocprofv3 record of the cfg4 iteration (tools/profile_train.sh ->
    profiles/<tag>_hbm_traffic.json with workload "cfg4 training iteration ...")."""
    import glob
    recs = [(json.load(open(f)), f) for f in glob.glob(os.path.join(ROOT, "profiles", "r*_hbm_traffic.json"))]
    for d, f in sorted(recs, key=lambda r: (r[0].get("created", ""), os.path.basename(r[1])), reverse=True):
        if (d.get("workload") or "").startswith("cfg4 training iteration"):
            return d, os.path.relpath(f, ROOT)
    return None, None


def train_roofline(live, stats, ms_iter, iters_timed_by_events):
    """The training leg's roofline (north_star: train iters/s "as fraction of HBM roofline").
    The iteration's dominant kernel is the composite's backward tile pass (k_render_bwd_mc<4,14>,
    a third of the iteration's kernel time): VALU-issue bound like the 3-channel pass, so
    `bound` = "valu" (committed PMC VALU count / live launch time against the spec issue rate),
    with its HBM view and the whole iteration's algorithmic bytes / ms_per_iter beside it."""
    rec, src = _pmc_train_record()
    ks = (rec or {}).get("kernels", {})
    kname = next((k for k in ks if k.startswith(TRAIN_DOM_KERNEL + "<")), None)
    kinfo = ks.get(kname, {}) if kname else {}
    ms_b, n_b = live.get("render_bwd_mc", (0.0, 0))
    ms_f, n_f = live.get("render_fwd_mc", (0.0, 0))
    t_b = ms_b / max(n_b, 1)
    B_iter, per_view, per_iter = train_algorithmic_bytes(**stats)
    peak = 1024 * VALU_CLOCK_GHZ / VALU_CYCLES_PER_INST
    b_launch = per_view["render_bwd_mc"]
    hbm = {"achieved": round(b_launch / (t_b * 1e-3) / 1e9, 1) if t_b > 0 else None, "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "bytes_per_launch": int(b_launch),
           "traffic": kinfo.get("traffic_bytes"), "traffic_source": src,
           "bytes": "SURVEY §8d render-backward bytes with the composite's 14 float channels (bench.py "
                    "train_algorithmic_bytes), measured R and P_v"}
    if hbm["achieved"] is not None:
        hbm["frac"] = round(hbm["achieved"] / HBM_PEAK_GBS, 5)
    _null_over_peak(hbm)
    pmc_iter = None
    if ks:
        n_iter = max((v.get("calls", 0) for k, v in ks.items() if k.startswith("k_adam")), default=0) or None
        if n_iter:
            pmc_iter = sum((v.get("traffic_bytes") or 0) * v["calls"] for v in ks.values()) / n_iter
    it = {"bytes": int(B_iter), "achieved": round(B_iter / (ms_iter * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
          "unit": "GB/s", "frac": round(B_iter / (ms_iter * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
          "per_view_bytes": {k: int(v) for k, v in per_view.items()},
          "per_iteration_bytes": {k: int(v) for k, v in per_iter.items()},
          "pmc_traffic_per_iter": None if pmc_iter is None else int(pmc_iter), "traffic_source": src,
          "what": "the iteration's algorithmic bytes (bench.py train_algorithmic_bytes) / ms_per_iter"}
    _null_over_peak(it)
    r = {"kernel": kname or TRAIN_DOM_KERNEL, "avg_launch_ms": round(t_b, 4), "launches": int(n_b),
         "render_fwd_mc_avg_launch_ms": round(ms_f / max(n_f, 1), 4),
         "launch_timing": f"HIP events on the launch stream around each composite tile pass, "
                          f"{iters_timed_by_events} iterations on one stream after the timed region (as "
                          "tools/train_kernels.py runs under rocprofv3)",
         "hbm": hbm, "iteration_hbm": it}
    if kinfo.get("valu_insts") and t_b > 0:
        ach = kinfo["valu_insts"] / (t_b * 1e-3) / 1e9
        r.update(bound="valu", achieved=round(ach, 1), peak=round(peak, 1), unit="Gwave-inst/s",
                 frac=round(ach / peak, 4), traffic=kinfo.get("traffic_bytes"),
                 valu_insts_per_launch=int(kinfo["valu_insts"]), valu_source=src,
                 peak_source="1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction (MI355X_MICROARCH.md)")
        if kinfo.get("salu_insts"):
            r["salu_insts_per_launch"] = int(kinfo["salu_insts"])
    else:
        r.update(bound="valu", achieved=None, peak=round(peak, 1), unit="Gwave-inst/s", frac=None,
                 traffic=kinfo.get("traffic_bytes"),
                 frac_null_reason="no committed rocprofv3 SQ_INSTS_VALU pass of the cfg4 iteration (profiles/)")
    return r


def train_leg(args, dev, dist, rank, world, backend, steps, warmup):
    """cfg4: the data-parallel relightable training iteration.  Every rank
    holds the whole scene (1.5M Gaussians: 1.36M foreground + 10 % sky on their (theta, phi)
    shell, cfg2 distribution, 1920x1080) and renders its own 4 views per iteration through the
    fused render(), with the reference's losses (L1 + D-SSIM, sky-BRDF, normal consistency,
    envlight, min-scale, sky depth) and backward; then one all-reduce of the flat gradient
    buffer, the densification statistics' SUM/MAX, and one fused Adam launch (gsr/train.py).
    The iteration number is past reg_normal_from_iter, so every loss term of train.py:77-118
    is on.  Returns the leg's numbers (iterations/s: whole job, weak scaling -- 4 views per
    rank per iteration; the time is the max over ranks)."""
    from gsr import train
    vpr = TRAIN_VIEWS_PER_RANK
    P_fg = args.P or 1_363_637
    W, H, focal = 1920, 1080, 1400.0
    scene, views, gts = train.synthetic_relit_scene(P_fg, vpr * world, W, H, focal, dev, seed=0)
    scene.iteration = TRAIN_ITERATION - 1
    mine = list(range(rank * vpr, (rank + 1) * vpr))
    my_views, my_gts = [views[i] for i in mine], [gts[i] for i in mine]
    ns = max(1, min(2 if args.streams is None else args.streams, vpr))
    streams = None if ns == 1 else [torch.cuda.Stream(dev) for _ in range(ns)]

    def step():
        return train.train_step(scene, my_views, mine, my_gts, world=world, streams=streams)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    ar_ms = None
    if dist is not None:
        t = torch.tensor([ms], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
        # the exchange step alone: the flat-gradient all-reduce
        for _ in range(3):
            dist.all_reduce(scene.fp.grad)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(10):
            dist.all_reduce(scene.fp.grad)
        torch.cuda.synchronize()
        ar_ms = (time.perf_counter() - t1) * 1e3 / 10
    # live launch times of the composite's tile passes for the roofline: a few iterations on
    # ONE stream after the timed region, the two passes bracketed by HIP events on their stream
    import diff_gaussian_rasterization as dgr
    from gsr import _lib
    ev_iters = max(1, args.event_steps)
    _lib.profile_read(reset=True)
    _lib.profile_stages(["render_fwd_mc", "render_bwd_mc"])
    _lib.profile_enable(True)
    for _ in range(ev_iters):
        train.train_step(scene, my_views, mine, my_gts, world=world, streams=None)
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    live = _lib.profile_read(reset=True)
    _lib.profile_stages(None)
    dgr.record_channels_calls(True)  # one more iteration for the measured R and P_v (after the events)
    train.train_step(scene, my_views, mine, my_gts, world=world, streams=None)
    dgr.record_channels_calls(False)
    stats = dict(P=scene.P, P_fg=P_fg, Pv=int(dgr.last_channels_call["visible"]), R=int(dgr.last_channels_call["num_rendered"]),
                 T=((W + 15) // 16) * ((H + 15) // 16), Npix=W * H, V=vpr, n_params=scene.fp.n)
    roof = train_roofline(live, stats, ms, ev_iters)
    return {"value": round(1e3 / ms, 3), "unit": "iters/s", "ms_per_iter": round(ms, 4), "steps": steps,
            "roofline": roof, "measured": {k: stats[k] for k in ("R", "Pv")},
            "warmup": warmup, "views_per_s": round(vpr * world * 1e3 / ms, 3),
            "workload": f"cfg4: {scene.P} Gaussians ({P_fg} fg + {scene.P - P_fg} sky), {W}x{H}, {vpr} views per "
                        f"GPU per iteration, env SH deg 4, sky SH deg 1, iteration {TRAIN_ITERATION} (every loss "
                        "term on)",
            "gaussians": scene.P, "views_per_iter": vpr * world, "streams": ns, "flat_params": scene.fp.n,
            "grad_bucket_mb": round(scene.fp.n * 4 / 1e6, 2),
            "grad_all_reduce_ms": None if ar_ms is None else round(ar_ms, 4),
            "all_reduce_backend": backend, "final_loss_rank0": round(float(loss) / vpr, 6)}


def bench_train(args, dev, dist, rank, world, backend, joined):
    """--config cfg4: the training iteration alone (train_leg) as the JSON line."""
    r = train_leg(args, dev, dist, rank, world, backend, args.steps, args.warmup)
    if rank == 0:
        print(json.dumps({
            "metric": "train iters/s (relit render + losses + backward + grad all-reduce + Adam, 4 views per GPU)",
            "value": r["value"], "unit": "iters/s", "n_gpus": world, "ranks_joined": joined, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": r["ms_per_iter"], "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": r["workload"], "gaussians": r["gaussians"], "width": 1920, "height": 1080,
                       "views_per_iter": r["views_per_iter"],
                       "parallelism": f"views x{world}" + (f" ({backend})" if backend else ""),
                       "flat_params": r["flat_params"], "streams": r["streams"]},
            "roofline": r["roofline"], "measured": r["measured"],
            "views_per_s": r["views_per_s"], "grad_all_reduce_ms": r["grad_all_reduce_ms"],
            "all_reduce_backend": backend, "grad_bucket_mb": r["grad_bucket_mb"],
            "final_loss_rank0": r["final_loss_rank0"]}), flush=True)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` (N > 1) started without a torch.distributed launcher around it:
    start the N rank processes here -- a `torch.distributed.run` child (one process per GPU,
    127.0.0.1 rendezvous) running this same command line -- relay their output, and fail
    unless the rank-0 line reports N ranks joined.  This process never touches the GPU
    (`import torch` does not initialise HIP), so the ranks own their devices."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "4"))
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True)
    line = None
    for ln in proc.stdout:
        sys.stdout.write(ln)
        sys.stdout.flush()
        if ln.startswith("{"):
            try:
                line = json.loads(ln)
            except ValueError:
                pass
    rc = proc.wait()
    if rc != 0:
        return rc
    if line is None or line.get("n_gpus") != n or line.get("ranks_joined") != n:
        got = None if line is None else (line.get("n_gpus"), line.get("ranks_joined"))
        print(f"bench.py: launched {n} ranks but the rank-0 line reports (n_gpus, ranks_joined) = {got}",
              file=sys.stderr)
        return 3
    return 0


def dist_setup(args):
    """(dist, rank, world, local, backend, ranks_joined) for this process.  One process per GPU
    over RCCL ("nccl"); GSR_DIST_BACKEND=gloo rehearses the N > 1 path (several ranks may then
    share a GPU: ranks wrap around the visible devices).  ranks_joined counts the processes
    that reached the first collective."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if world == 1:
        return None, 0, 1, local, None, 1
    import torch.distributed as dist
    backend = os.environ.get("GSR_DIST_BACKEND", "nccl")
    if args.launch_probe:  # CPU-only check of the launcher (tests/test_bench_launch.py)
        backend = "gloo"
        dist.init_process_group("gloo")
        one = torch.ones(1)
    else:
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        one = torch.ones(1, device=torch.device("cuda", local))
    dist.all_reduce(one)
    return dist, rank, world, local, backend, int(one.item())


def clustered_leg(args, dev, name="cfg2c", V=4, NS=3):
    """The headline's size on a Trevi-class clustered cloud (gsr.scenes.trevi_like_gaussians:
    facade sheets with a density gradient, sculpture clusters, a translucent spray volume, the
    reference's sky band; ~20 % culled, heavy tiles).  Reports the §8d single call (median of 50),
    the 4-view / 3-stream throughput the headline uses, stage_ms over STAGE_VIEWS one-stream
    views and the dominant stage's roofline (PMC record of `bench.py --config cfg2c`)."""
    from diff_gaussian_rasterization import _C
    from gsr import _lib, scenes
    cam, gs_cpu, cfg = scenes.build_config(name, device="cpu", seed=0)
    W, H, deg = cam.image_width, cam.image_height, cfg["sh_degree"]
    g = {k: v.to(dev) for k, v in gs_cpu.items() if k != "is_sky"}
    P, M = g["means3D"].shape[0], g["shs"].shape[1]
    e = torch.empty(0, device=dev)
    bg = torch.zeros(3, device=dev)
    dout = torch.randn(3, H, W, generator=torch.Generator().manual_seed(1)).to(dev)
    cams = [scenes.view_camera(cam, k, look=cfg.get("look")).to(dev) for k in range(V)]
    mats = [(c.world_view_transform, c.full_proj_transform, c.camera_center) for c in cams]
    state = {}

    def view(k=0):
        vm, pm, cp = mats[k]
        R, color, radii, geom, binb, img = _C.rasterize_gaussians(
            bg, g["means3D"], e, g["opacities"], g["scales"], g["rotations"], 1.0, e, vm, pm, cam.tanfovx,
            cam.tanfovy, H, W, g["shs"], deg, cp, False)
        _C.rasterize_gaussians_backward(bg, g["means3D"], radii, e, g["scales"], g["rotations"], 1.0, e, vm, pm,
                                        cam.tanfovx, cam.tanfovy, dout, g["shs"], deg, cp, geom, R, binb, img)
        if k == 0:
            state["R"], state["radii"] = R, radii

    main_s = torch.cuda.current_stream(dev)
    ss = [torch.cuda.Stream(dev) for _ in range(NS)]

    def step():
        for s_ in ss:
            s_.wait_stream(main_s)
        for i in range(V):
            with torch.cuda.stream(ss[i % NS]):
                view(i)
        for s_ in ss:
            main_s.wait_stream(s_)

    view()
    torch.cuda.synchronize()
    stages = stage_breakdown(view, STAGE_VIEWS)
    dom_name = max(((k, v[0] / v[1]) for k, v in stages.items() if v[1] > 0 and k in STAGE_KERNEL),
                   key=lambda kv: kv[1])[0]
    single = single_call_median(view, W, H)
    for _ in range(SETTLE_STEPS):
        step()
    torch.cuda.synchronize()
    nsteps = max(5, args.steps)
    t0 = time.perf_counter()
    for _ in range(nsteps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / nsteps
    _lib.profile_stages([dom_name])
    _lib.profile_enable(True)
    for _ in range(max(1, args.event_steps)):
        for i in range(V):
            view(i)
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    live = _lib.profile_read(reset=True).get(dom_name, (0.0, 0))
    _lib.profile_stages(None)
    R, Pv = int(state["R"]), int((state["radii"] > 0).sum().item())
    T = ((W + 15) // 16) * ((H + 15) // 16)
    workload = f"{name}: {P} Gaussians SH{deg}, {W}x{H}"
    roof = tile_roofline((dom_name, live[0] / max(live[1], 1)), P, Pv, R, T, W, H, M, workload, dev)
    return {"value": round(V * W * H / (ms * 1e-3) / 1e6, 3), "unit": "MPix/s", "ms_per_step": round(ms, 4),
            "steps": nsteps, "views_per_step": V, "streams": NS, "single_call": single,
            "stage_ms": {k: round(v[0] / max(v[1], 1), 4) for k, v in stages.items() if v[1] > 0},
            "stage_views": STAGE_VIEWS, "roofline": roof,
            "measured": {"num_rendered": R, "visible": Pv, "culled_frac": round(1 - Pv / P, 4)},
            "config": {"workload": workload + ": Trevi-class clustered cloud (gsr.scenes.trevi_like_gaussians: "
                                              "facade sheets, sculpture clusters, translucent spray, side "
                                              "buildings, 10 % sky band as augment_with_sky_gaussians), "
                                              f"{V} views per step on {NS} HIP streams",
                       "gaussians": P, "width": W, "height": H, "sh_degree": deg}}


def refalgo_leg(args, bg, g, e, vm, pm, cp, cam, H, W, deg, dout, ms_ours):
    """The reference rasterizer's stage structure in plain HIP on the same GPU and inputs
    (baseline/refalgo.hip: 64-bit duplicate keys + hipcub radix sort, one thread per pixel,
    9 global atomics per (pixel, Gaussian) in the backward).  Timed after, not inside, the
    timed region; `speedup` = its step time / libgsr's."""
    from baseline.refalgo import RefAlgoRasterizer
    ras = RefAlgoRasterizer()

    def step():
        R, color, radii = ras.forward(bg, g["means3D"], e, g["opacities"], g["scales"], g["rotations"], 1.0, e, vm,
                                      pm, cam.tanfovx, cam.tanfovy, H, W, g["shs"], deg, cp)
        ras.backward(bg, g["means3D"], radii, g["scales"], g["rotations"], 1.0, e, vm, pm, cam.tanfovx, cam.tanfovy,
                     dout, g["shs"], deg, cp)

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    n = max(1, min(args.steps, 10))
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / n
    return {"value": round(W * H / (ms * 1e-3) / 1e6, 3), "unit": "MPix/s", "ms_per_step": round(ms, 4),
            "steps": n, "speedup": round(ms / ms_ours, 3),
            "what": "reference stage structure in plain HIP on this MI355X (baseline/refalgo.hip): per-Gaussian "
                    "preprocess, hipcub inclusive scan + D2H num_rendered, duplicateWithKeys (64-bit tile|depth "
                    "keys), hipcub radix sort on 32+msb(T) bits, tile ranges, 16x16-thread per-pixel render with "
                    "256-Gaussian shared-memory rounds, per-pixel backward with 9 global atomics per pair; shares "
                    "libgsr's per-Gaussian preprocess kernels (so it is an upper bound on the reference's speed)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one rank process each); N > 1 without WORLD_SIZE in the environment starts the N "
                         "ranks itself (torch.distributed.run child, 127.0.0.1 rendezvous)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--P", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-tiles", type=int, default=64)
    ap.add_argument("--ply", default=None, help="a trained scene (GaussianModel.save_ply layout) instead of cfg2's "
                                               "synthetic cloud; camera looks at the foreground's median from "
                                               "2x its extent, 1920x1080, focal 1400")
    ap.add_argument("--colmap", default=None, help="with --ply: a NeRF-OSR / COLMAP scene folder (sparse/0 model); "
                                                  "renders from its training camera --view at the reference's "
                                                  "default resolution rule")
    ap.add_argument("--view", type=int, default=0)
    ap.add_argument("--fused-only", action="store_true", help="cfg3: time only the fused render()")
    ap.add_argument("--views-per-step", "--views-per-sync", dest="views_per_step", type=int, default=None,
                    help="views per step per GPU (default 4 at every N: the per-GPU mini-batch whose gradients "
                         "cross the ranks in one all-reduce at N > 1)")
    ap.add_argument("--streams", type=int, default=None,
                    help="HIP streams the views of a step (cfg2 / cfg2c, default 3) or a training iteration "
                         "(cfg4, default 2) alternate over")
    ap.add_argument("--no-minibatch", action="store_true", help="skip the 4-view multi-stream extra leg")
    ap.add_argument("--no-refalgo", action="store_true", help="skip the reference-structure GPU baseline leg")
    ap.add_argument("--no-clustered", action="store_true",
                    help="skip the cfg2c leg (cfg2's size on a Trevi-class clustered cloud)")
    ap.add_argument("--no-relit", action="store_true", help="skip the cfg3 / cfg5-relit relight legs of the default line")
    ap.add_argument("--event-steps", type=int, default=5,
                    help="steps (each V views, one stream) run after the timed region with the dominant stage's "
                         "HIP events, for roofline.avg_launch_ms (default 5); the timed region carries no events")
    ap.add_argument("--no-train", action="store_true", help="skip the cfg4 training-iteration leg (train iters/s)")
    ap.add_argument("--train-steps", type=int, default=None, help="timed iterations of the training leg "
                                                                  "(default min(--steps, 20))")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N > 1: all-reduce each step's gradient bucket before the next step starts (default: the "
                         "exchange of step i runs on the collective stream under step i+1's views)")
    ap.add_argument("--launch-probe", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    dist, rank, world, local, backend, joined = dist_setup(args)
    if args.launch_probe:
        if rank == 0:
            print(json.dumps({"metric": "launch probe", "n_gpus": world, "ranks_joined": joined,
                              "backend": backend}), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if args.config in ("cfg3", "cfg5-relit"):
        bench_relight(args, dev)
        return
    if args.config == "cfg4":
        bench_train(args, dev, dist, rank, world, backend, joined)
        if dist is not None:
            dist.destroy_process_group()
        return

    from diff_gaussian_rasterization import _C
    from gsr import _lib, scenes
    from gsr import dp as gdp

    if args.ply:
        cam, gs_cpu, cfg = scenes.ply_config(args.ply)
        if args.colmap:
            from gsr import colmap as gcm
            train, _, _ = gcm.read_nerf_osr_info(args.colmap)
            cam = gcm.render_camera(train[args.view % len(train)])
            cfg = dict(cfg, W=cam.image_width, H=cam.image_height)
    else:
        # one scene replicated on every rank (the data-parallel replica); the ranks differ in views
        cam, gs_cpu, cfg = scenes.build_config(args.config, device="cpu", seed=0, P=args.P)
    W, H, deg = cam.image_width, cam.image_height, cfg["sh_degree"]
    P = gs_cpu["means3D"].shape[0]
    g = {k: v.to(dev) for k, v in gs_cpu.items()}
    M = g["shs"].shape[1]
    e = torch.empty(0, device=dev)
    bg = torch.zeros(3, device=dev)
    gen = torch.Generator().manual_seed(1)
    dout_cpu = torch.randn(3, H, W, generator=gen)
    dout = dout_cpu.to(dev)
    # V views per step per rank, 4 by default at every N (cfg4's per-GPU mini-batch, whose
    # gradients accumulate into one bucket and cross the ranks in ONE RCCL all-reduce at N > 1;
    # the same per-rank work at every N).  Rank r renders global views r*V .. r*V+V-1 of the scene.
    V = max(1, args.views_per_step if args.views_per_step is not None else 4)
    # the step's views alternate over NS HIP streams (default 3): one view's latency-bound
    # geometry passes overlap another's tile passes
    NS = max(1, min(3 if args.streams is None else args.streams, V))
    cams = [scenes.view_camera(cam, rank * V + k, look=cfg.get("look")).to(dev) for k in range(V)]
    mats = [(c.world_view_transform, c.full_proj_transform, c.camera_center) for c in cams]
    main_s = torch.cuda.current_stream(dev)
    vstreams = [main_s] if NS == 1 else [torch.cuda.Stream(dev) for _ in range(NS)]
    state = {}

    def view(k=0):
        """One rasterizer forward + backward through the drop-in _C (the reference's call pair)."""
        vm, pm, cp = mats[k]
        R, color, radii, geom, binb, img = _C.rasterize_gaussians(
            bg, g["means3D"], e, g["opacities"], g["scales"], g["rotations"], 1.0, e, vm, pm, cam.tanfovx,
            cam.tanfovy, H, W, g["shs"], deg, cp, False)
        grads = _C.rasterize_gaussians_backward(bg, g["means3D"], radii, e, g["scales"], g["rotations"], 1.0, e, vm,
                                                pm, cam.tanfovx, cam.tanfovy, dout, g["shs"], deg, cp, geom, R, binb,
                                                img)
        if k == 0:
            state["R"], state["radii"] = R, radii
        return grads

    overlap = dist is not None and not args.no_overlap
    state["k"], state["work"] = 0, [None, None]

    def drain():
        """Wait (on the current stream) for every exchange still in flight."""
        for j, w in enumerate(state["work"]):
            if w is not None:
                w.wait()
                state["work"][j] = None

    def step():
        """V views, one after another (or alternating over NS HIP streams with --streams).  At
        N > 1 the views' dL/d(means3D, sh, opacity, scales, rotations) are summed into one flat
        bucket on the main stream and over the ranks with one all-reduce.  Two buckets
        alternate: step i's all-reduce is issued asynchronously (the collective's own stream
        waits for the bucket) and runs under step i+1's views; a bucket is refilled only after
        its previous exchange has finished (work.wait orders the stream after it)."""
        kb = state["k"] % (2 if overlap else 1)
        if dist is not None and state["work"][kb] is not None:
            state["work"][kb].wait()
            state["work"][kb] = None
        for s in vstreams:
            if s is not main_s:
                s.wait_stream(main_s)  # the bucket's previous exchange comes first
        for i in range(V):
            s = vstreams[i % NS]
            with torch.cuda.stream(s):
                grads = view(i)
            if dist is not None:
                ts = [grads[3], grads[5], grads[2], grads[6], grads[7]]
                if s is not main_s:
                    main_s.wait_stream(s)
                    for t in ts:
                        t.record_stream(main_s)
                if "buckets" not in state:
                    state["buckets"] = [gdp.GradBucket(ts) for _ in range(2 if overlap else 1)]
                b = state["buckets"][kb]
                if i == 0:
                    b.pack(ts)
                else:
                    for v, t in zip(b.views(), ts):
                        v.add_(t)
        for s in vstreams:
            if s is not main_s:
                main_s.wait_stream(s)
        if dist is not None:
            state["work"][kb] = dist.all_reduce(state["buckets"][kb].flat, async_op=True)
            if not overlap:
                drain()
        state["k"] += 1

    step()  # first-call setup (allocations, the speculative binning's sizes)
    drain()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    # Stage breakdown (before the W warmup steps, so the timed region follows them directly
    # and starts on a busy GPU's clocks): three profiled views, one at a time on one stream
    # (every stage bracketed by HIP events).  The timed region carries no events; the dominant
    # stage's launch time comes from --event-steps steps on one stream after it.
    stages = stage_breakdown(view, STAGE_VIEWS)
    dom_name = max(((k, v[0] / v[1]) for k, v in stages.items() if v[1] > 0 and k in STAGE_KERNEL),
                   key=lambda kv: kv[1])[0]
    # at least SETTLE_STEPS untimed steps in a row before the timed region (the W warmup steps
    # plus settle steps): with 3 warmup steps a 10-step run read ~1 % slower than with 20
    settle = max(0, SETTLE_STEPS - args.warmup)
    for _ in range(settle + args.warmup):
        step()
    drain()  # the timed region starts with no exchange in flight ...
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()  # ... and ends with every step's exchange finished
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    # the dominant stage's live launch time: --event-steps steps' views one after another on ONE
    # stream, that stage bracketed by HIP events on the stream it launches on (in the timed
    # region the views overlap on NS streams, which would fold the other streams' kernels into
    # a launch's duration); tools/profile_round.sh profiles the same one-stream layout
    _lib.profile_stages([dom_name])
    _lib.profile_enable(True)
    ev_steps = max(1, args.event_steps)
    for _ in range(ev_steps):
        for i in range(V):
            view(i)
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    live = _lib.profile_read(reset=True).get(dom_name, (0.0, 0))
    _lib.profile_stages(None)
    ms = (t1 - t0) * 1e3 / args.steps
    if dist is not None:
        t = torch.tensor([ms], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())

    ar_ms = None
    if dist is not None:
        for _ in range(2):
            state["buckets"][0].all_reduce()
        torch.cuda.synchronize()
        ta = time.perf_counter()
        for _ in range(5):
            state["buckets"][0].all_reduce()
        torch.cuda.synchronize()
        ar_ms = (time.perf_counter() - ta) * 1e3 / 5
    R = int(state["R"])
    Pv = int((state["radii"] > 0).sum().item())
    T = ((W + 15) // 16) * ((H + 15) // 16)
    per_stage = {k: round(v[0] / max(v[1], 1), 4) for k, v in stages.items() if v[1] > 0}
    dom = (dom_name, live[0] / max(live[1], 1))

    single = mini = None
    if rank == 0 and world == 1:
        # SURVEY §8d's definition: W*H / (t_fwd + t_bwd) of ONE call, the median of >= 50 calls
        # after 10 warm-up, HIP events on the stream the calls run on
        single = single_call_median(view, W, H)
        if not args.no_minibatch and not (V == 4 and NS == 3):  # (the timed step already is this layout)
            # a 4-view mini-batch of DISTINCT cameras on 3 HIP streams: one view's latency-bound
            # geometry passes overlap another's tile passes (throughput, not the reference's pattern)
            mcams = [scenes.view_camera(cam, k, look=cfg.get("look")).to(dev) for k in range(4)]
            mm = [(c.world_view_transform, c.full_proj_transform, c.camera_center) for c in mcams]
            ss = [torch.cuda.Stream(dev) for _ in range(3)]
            saved = list(mats)
            mats[:] = mm + mats[len(mm):] if len(mats) >= len(mm) else mm

            def mstep():
                for s_ in ss:
                    s_.wait_stream(main_s)
                for i in range(4):
                    with torch.cuda.stream(ss[i % 3]):
                        view(i)
                for s_ in ss:
                    main_s.wait_stream(s_)

            for _ in range(3):
                mstep()
            torch.cuda.synchronize()
            tm = time.perf_counter()
            nm = max(5, min(args.steps, 20))
            for _ in range(nm):
                mstep()
            torch.cuda.synchronize()
            mms = (time.perf_counter() - tm) * 1e3 / nm
            mats[:] = saved
            mini = {"ms_per_4_views": round(mms, 4), "value": round(4 * W * H / (mms * 1e-3) / 1e6, 3),
                    "unit": "MPix/s", "what": "4 distinct cameras of the same scene per step, alternating over 3 "
                                              "HIP streams"}
    workload = (f"ply {os.path.basename(args.ply)}" if args.ply else args.config) + f": {P} Gaussians SH{deg}, {W}x{H}"
    roofline = tile_roofline(dom, P, Pv, R, T, W, H, M, workload, dev)
    out = {
        "metric": METRIC, "value": round(world * V * W * H / (ms * 1e-3) / 1e6, 3), "unit": "MPix/s",
        "n_gpus": world, "ranks_joined": joined, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic", "untimed_steps_before_timing": settle + args.warmup,
        "config": {"workload": (f"ply {os.path.basename(args.ply)}" + (f" + COLMAP view {args.view}" if args.colmap
                                                                       else "") if args.ply else args.config)
                               + f": {P} Gaussians SH{deg}, {W}x{H}, one rasterizer forward + backward per view, "
                                 f"{V} view(s) per step per GPU"
                               + (f" on {NS} HIP streams" if NS > 1 else "")
                               + (f", scene replicated on every rank, distinct cameras per rank, one {backend} "
                                  "grad all-reduce per step" + (" (overlapped with the next step's views)" if overlap
                                                                else "") if world > 1 else ""),
                   "gaussians": P, "width": W, "height": H, "sh_degree": deg, "num_rendered": R, "visible": Pv,
                   "views_per_step": V, "streams": NS,
                   "parallelism": f"views x{world}" + (f" ({backend})" if backend else "")},
        "roofline": roofline,
        "stage_ms": per_stage,
        "stage_ms_source": f"{STAGE_VIEWS} views one at a time on one stream before the timed region (HIP events around every "
                           "stage); roofline.avg_launch_ms is the dominant stage's events over "
                           f"{ev_steps} steps' views run one at a time on one stream right after the timed region",
    }
    if single is not None:
        out["single_call"] = single
    if mini is not None:
        out["minibatch_4view"] = mini
    if dist is not None:
        out["data_parallel"] = {"views_per_step": V, "backend": backend, "grad_all_reduce_ms": round(ar_ms, 4),
                                "grad_all_reduce_what": "the step's bucket all-reduced alone, 5 times back to back",
                                "exchange_overlapped": overlap,
                                "grad_bucket_mb": round(state["buckets"][0].flat.numel() * 4 / 1e6, 2)}
    if not args.no_train and not args.ply:
        # the metric's second half: train iters/s of the cfg4 iteration at this N
        state.pop("buckets", None)
        out["train"] = train_leg(args, dev, dist, rank, world, backend,
                                 args.train_steps or min(args.steps, 20), max(3, min(args.warmup, 10)))
    if rank == 0 and world == 1 and args.config == "cfg2" and not args.no_clustered and not args.ply:
        # the same size on a Trevi-class clustered cloud (culling, heavy tiles, sky band)
        out["clustered"] = clustered_leg(args, dev)
        torch.cuda.empty_cache()
        if single is not None and out["clustered"].get("single_call"):
            # SURVEY §8d's definition figure (one forward + backward call pair, 1.5M Gaussians at
            # 1080p) on both clouds side by side: the uniform cfg2 and the Trevi-class cfg2c
            cs = out["clustered"]["single_call"]
            out["single_call_definition"] = {
                "cfg2_ms": single["median_ms"], "cfg2c_ms": cs["median_ms"],
                "cfg2_mpix_per_s": round(W * H / (single["median_ms"] * 1e-3) / 1e6, 1),
                "cfg2c_mpix_per_s": round(W * H / (cs["median_ms"] * 1e-3) / 1e6, 1),
                "what": "median of 50 isolated call pairs (bench.py single_call_median); `value` is the 4-view "
                        "3-stream throughput"}
    if rank == 0 and world == 1 and not args.no_relit and not args.ply:
        # BASELINE configs[2] and configs[4] at their sizes, timed by the same run: the relight
        # render with backward (cfg3: 1M + 0.1M sky Gaussians at 1080p; cfg5: 4.55M + 0.45M at 4K)
        rl = {}
        for key, stress in (("cfg3", False), ("cfg5_relit", True)):
            r = relight_leg(args, dev, stress, 10, 3, with_calls=False, P_fg=4_545_455 if stress else 1_000_000)
            rl[key] = {k: r[k] for k in ("value", "unit", "ms_per_step", "steps", "warmup", "mpix_per_s", "config",
                                          "roofline", "measured", "implementation", "loss")}
            torch.cuda.empty_cache()
        out["relit"] = rl
    if rank == 0 and world == 1 and not args.no_refalgo and not args.ply:
        ms_view = single["median_ms"] if single is not None else ms / V
        vm, pm, cp = mats[0]
        out["gpu_reference_algorithm"] = refalgo_leg(args, bg, g, e, vm, pm, cp, cam, H, W, deg, dout, ms_view)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(cam, gs_cpu, deg, dout_cpu, ntiles=args.cpu_tiles)
        out["cpu_baseline"] = {k: (round(v, 6) if isinstance(v, float) else v) for k, v in cb.items()}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()

if __name__ == "__main__":
    main()
