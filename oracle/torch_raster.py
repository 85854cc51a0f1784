"""oracle/torch_raster.py -- TEST INFRASTRUCTURE / CPU BASELINE ONLY.

The north star's "naive PyTorch-CPU rasterizer" (BASELINE.json, SURVEY §8d "CPU
baseline"): the reference's algorithm written with PyTorch CPU ops, vectorised over
Gaussians in the per-Gaussian stages and over (tile, pixel) in the tile passes, run on all
the host cores PyTorch is given.  bench.py's `cpu_baseline` leg times it; tests check it
against the C oracle (tests/test_torch_raster_cpu.py).  The product path never imports it.

Follows, stage by stage:
  preprocess   forward.cu:155-256 (+ computeCov3D :118-152, computeCov2D :74-113,
               computeColorFromSH :20-71, in_frustum auxiliary.h:139-164, getRect :46-56,
               ndc2Pix :41-44 in double)
  binning      rasterizer_impl.cu:70-111 duplicateWithKeys (key = tile << 32 | depth bits),
               :300-308 stable radix sort (torch.sort(stable=True) on the 64-bit keys),
               :116-138 identifyTileRanges
  render fwd   forward.cu:261-374 renderCUDA: the per-pixel loop over a tile's list, here
               one step per list position for a batch of tiles at once ([tiles, 256] pixels)
  render bwd   backward.cu:399-557 renderCUDA backward, back to front, same recurrences,
               per-(tile, Gaussian) sums scattered with index_add_ (the reference's atomics)
  preproc bwd  backward.cu:144-396 (computeCov2DCUDA + preprocessCUDA backward): autograd
               through the differentiable preprocess (the same derivative: the screen-space
               mean gradient arrives in NDC units, the conic's off-diagonal gradient is the
               reference's symmetric half, so it is doubled before it enters autograd).
"""
import torch

BLOCK = 16
SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
SH_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435)


def _sh_rgb(deg, sh, dirs):
    """computeColorFromSH (forward.cu:20-71): sh [P, M, 3], dirs [P, 3] unit -> [P, 3] before +0.5."""
    res = SH_C0 * sh[:, 0]
    if deg > 0:
        x, y, z = dirs[:, 0:1], dirs[:, 1:2], dirs[:, 2:3]
        res = res - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            res = (res + SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5] + SH_C2[2] * (2.0 * zz - xx - yy) * sh[:, 6]
                   + SH_C2[3] * xz * sh[:, 7] + SH_C2[4] * (xx - yy) * sh[:, 8])
            if deg > 2:
                res = (res + SH_C3[0] * y * (3.0 * xx - yy) * sh[:, 9] + SH_C3[1] * xy * z * sh[:, 10]
                       + SH_C3[2] * y * (4.0 * zz - xx - yy) * sh[:, 11]
                       + SH_C3[3] * z * (2.0 * zz - 3.0 * xx - 3.0 * yy) * sh[:, 12]
                       + SH_C3[4] * x * (4.0 * zz - xx - yy) * sh[:, 13] + SH_C3[5] * z * (xx - yy) * sh[:, 14]
                       + SH_C3[6] * x * (xx - 3.0 * yy) * sh[:, 15])
    return res


def preprocess(means3D, scales, rotations, opacities, shs, deg, viewmatrix, projmatrix, campos, W, H, tanfovx,
               tanfovy, scale_modifier=1.0, colors=None):
    """Differentiable preprocess of all P Gaussians.  Returns a dict with `ndc` [P,2] (the
    quantity whose gradient the reference calls dL_dmean2D), `xy` [P,2] pixel centres,
    `conic` [P,3] (a, b, c), `rgb` [P,3], `depth` [P], `radii` [P] int, `rect` [P,4]
    (xmin, ymin, xmax, ymax in tiles), `tiles` [P]; culled Gaussians have radii 0."""
    vm, pm = viewmatrix.reshape(4, 4), projmatrix.reshape(4, 4)
    P = means3D.shape[0]
    ones = torch.ones(P, 1, dtype=means3D.dtype)
    ph = torch.cat([means3D, ones], 1)
    t = ph @ vm  # row vector x row-major matrix (auxiliary.h:58-77)
    hom = ph @ pm
    pw = 1.0 / (hom[:, 3:4] + 1e-7)
    ndc = hom[:, 0:2] * pw
    # cov3D (quaternion as given)
    s = scale_modifier * scales
    r, x, y, z = rotations.unbind(1)
    R = torch.stack([torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], 1),
                     torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], 1),
                     torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], 1)], 1)
    # glm: M = S * R with R's constructor taking columns -> M[row][col] = s[row] * R_given[col][row]
    Mm = s[:, :, None] * R.transpose(1, 2)
    Sigma = Mm.transpose(1, 2) @ Mm
    # cov2D (EWA, with the +-1.3 tan clamp)
    focal_x = W / (2.0 * tanfovx)
    focal_y = H / (2.0 * tanfovy)
    tz = t[:, 2]
    limx, limy = 1.3 * tanfovx, 1.3 * tanfovy
    tx = torch.clamp(t[:, 0] / tz, -limx, limx) * tz
    ty = torch.clamp(t[:, 1] / tz, -limy, limy) * tz
    zero = torch.zeros_like(tz)
    J = torch.stack([torch.stack([focal_x / tz, zero, -(focal_x * tx) / (tz * tz)], 1),
                     torch.stack([zero, focal_y / tz, -(focal_y * ty) / (tz * tz)], 1)], 1)  # [P,2,3]
    Wv = vm[:3, :3].T  # rows of the view rotation
    Tm = J @ Wv  # [P,2,3]
    cov = Tm @ Sigma @ Tm.transpose(1, 2)
    a = cov[:, 0, 0] + 0.3
    b = cov[:, 0, 1]
    c = cov[:, 1, 1] + 0.3
    det = a * c - b * b
    ok = (t[:, 2] > 0.2) & (det != 0)
    det_safe = torch.where(ok, det, torch.ones_like(det))
    det_inv = 1.0 / det_safe
    conic = torch.stack([c * det_inv, -b * det_inv, a * det_inv], 1)
    with torch.no_grad():
        mid = 0.5 * (a + c)
        l1 = mid + torch.sqrt(torch.clamp(mid * mid - det, min=0.1))
        l2 = mid - torch.sqrt(torch.clamp(mid * mid - det, min=0.1))
        radius = torch.ceil(3.0 * torch.sqrt(torch.maximum(l1, l2)))
        radius = torch.where(ok, radius, torch.zeros_like(radius))
        nd = ndc.detach().double()
        px = (((nd[:, 0] + 1.0) * W - 1.0) * 0.5).float()
        py = (((nd[:, 1] + 1.0) * H - 1.0) * 0.5).float()
        gx, gy = (W + BLOCK - 1) // BLOCK, (H + BLOCK - 1) // BLOCK
        ri = radius.to(torch.int64)
        rf = ri.float()
        xmin = ((px - rf) / BLOCK).to(torch.int64).clamp(0, gx)
        ymin = ((py - rf) / BLOCK).to(torch.int64).clamp(0, gy)
        xmax = (((px + rf) + BLOCK - 1) / BLOCK).to(torch.int64).clamp(0, gx)
        ymax = (((py + rf) + BLOCK - 1) / BLOCK).to(torch.int64).clamp(0, gy)
        tiles = (xmax - xmin) * (ymax - ymin)
        vis = ok & (tiles > 0)
        radii = torch.where(vis, ri, torch.zeros_like(ri)).to(torch.int32)
        tiles = torch.where(vis, tiles, torch.zeros_like(tiles))
    if colors is None:
        d = means3D - campos.reshape(1, 3)
        d = d / torch.sqrt((d * d).sum(1, keepdim=True))
        rgb = torch.clamp_min(_sh_rgb(deg, shs, d) + 0.5, 0.0)
    else:
        rgb = colors
    return dict(ndc=ndc, xy=torch.stack([px, py], 1), conic=conic, rgb=rgb, depth=t[:, 2].detach(), radii=radii,
                rect=torch.stack([xmin, ymin, xmax, ymax], 1), tiles=tiles, opacity=opacities.reshape(-1))


def binning(pre, W, H):
    """duplicateWithKeys + stable sort + identifyTileRanges: (point_list [R], ranges [T,2])."""
    gx, gy = (W + BLOCK - 1) // BLOCK, (H + BLOCK - 1) // BLOCK
    T = gx * gy
    tiles = pre["tiles"]
    vis = torch.nonzero(tiles > 0).reshape(-1)
    cnt = tiles[vis]
    R = int(cnt.sum())
    if R == 0:
        return torch.zeros(0, dtype=torch.int64), torch.zeros(T, 2, dtype=torch.int64)
    gid = torch.repeat_interleave(vis, cnt)
    first = torch.repeat_interleave(torch.cumsum(cnt, 0) - cnt, cnt)
    k = torch.arange(R, dtype=torch.int64) - first  # instance index within its Gaussian
    rect = pre["rect"][gid]
    w = rect[:, 2] - rect[:, 0]
    tx = rect[:, 0] + k % w  # y outer, x inner (rasterizer_impl.cu:92-103)
    ty = rect[:, 1] + k // w
    tile = ty * gx + tx
    dbits = pre["depth"].contiguous().view(torch.int32).to(torch.int64)[gid] & 0xFFFFFFFF
    keys = (tile << 32) | dbits
    _, order = torch.sort(keys, stable=True)
    point_list = gid[order]
    tsorted = tile[order]
    counts = torch.bincount(tsorted, minlength=T)
    ends = torch.cumsum(counts, 0)
    ranges = torch.stack([ends - counts, ends], 1)
    ranges[counts == 0] = 0
    return point_list, ranges


def _tile_batch(tiles, ranges, point_list, W, gx):
    L = (ranges[tiles, 1] - ranges[tiles, 0])
    Lmax = int(L.max()) if tiles.numel() else 0
    pos = torch.arange(Lmax, dtype=torch.int64)[None, :]
    idx = ranges[tiles, 0][:, None] + pos
    valid = pos < L[:, None]
    ids = torch.where(valid, point_list[idx.clamp(max=max(point_list.numel() - 1, 0))], torch.zeros_like(idx))
    lx = torch.arange(BLOCK * BLOCK) % BLOCK
    ly = torch.arange(BLOCK * BLOCK) // BLOCK
    px = (tiles % gx)[:, None] * BLOCK + lx[None, :]
    py = (tiles // gx)[:, None] * BLOCK + ly[None, :]
    return ids, valid, L, px, py


def render_fwd(tiles, ranges, point_list, xy, conic, opacity, feat, bg, W, H):
    """renderCUDA forward for the given tiles: (color [nt,256,3], final_T [nt,256],
    n_contrib [nt,256], inside [nt,256])."""
    gx = (W + BLOCK - 1) // BLOCK
    ids, valid, L, px, py = _tile_batch(tiles, ranges, point_list, W, gx)
    inside = (px < W) & (py < H)
    pxf, pyf = px.float(), py.float()
    nt = tiles.numel()
    Tr = torch.ones(nt, BLOCK * BLOCK)
    C = torch.zeros(nt, BLOCK * BLOCK, 3)
    done = ~inside
    last = torch.zeros(nt, BLOCK * BLOCK, dtype=torch.int64)
    for j in range(ids.shape[1]):
        g = ids[:, j]
        dx = xy[g, 0:1] - pxf
        dy = xy[g, 1:2] - pyf
        co = conic[g]
        power = -0.5 * (co[:, 0:1] * dx * dx + co[:, 2:3] * dy * dy) - co[:, 1:2] * dx * dy
        alpha = torch.clamp(opacity[g][:, None] * torch.exp(power), max=0.99)
        ok = valid[:, j:j + 1] & ~done & (power <= 0) & (alpha >= 1.0 / 255.0)
        test_T = Tr * (1 - alpha)
        sat = ok & (test_T < 0.0001)
        done = done | sat
        ok = ok & ~sat
        w = torch.where(ok, alpha * Tr, torch.zeros_like(Tr))
        C = C + feat[g][:, None, :] * w[:, :, None]
        Tr = torch.where(ok, test_T, Tr)
        last = torch.where(ok, torch.full_like(last, j + 1), last)
    color = C + Tr[:, :, None] * bg.reshape(1, 1, 3)
    return color, Tr, last, inside


def render_bwd(P, tiles, ranges, point_list, xy, conic, opacity, feat, bg, final_T, n_contrib, dL_dpix, W, H):
    """renderCUDA backward for the given tiles (dL_dpix [nt,256,3]): per-Gaussian
    dL_dmean2D [P,3] (NDC units), dL_dconic [P,2,2], dL_dopacity [P,1], dL_dcolors [P,3]."""
    gx = (W + BLOCK - 1) // BLOCK
    ids, valid, L, px, py = _tile_batch(tiles, ranges, point_list, W, gx)
    inside = (px < W) & (py < H)
    pxf, pyf = px.float(), py.float()
    g_mean = torch.zeros(P, 3)
    g_conic = torch.zeros(P, 2, 2)
    g_op = torch.zeros(P, 1)
    g_col = torch.zeros(P, 3)
    Tr = final_T.clone()
    accum = torch.zeros_like(dL_dpix)
    last_alpha = torch.zeros_like(Tr)
    last_color = torch.zeros_like(dL_dpix)
    bg_dot = (dL_dpix * bg.reshape(1, 1, 3)).sum(-1)
    for j in range(ids.shape[1] - 1, -1, -1):
        g = ids[:, j]
        act = valid[:, j:j + 1] & inside & (j < n_contrib)
        dx = xy[g, 0:1] - pxf
        dy = xy[g, 1:2] - pyf
        co = conic[g]
        power = -0.5 * (co[:, 0:1] * dx * dx + co[:, 2:3] * dy * dy) - co[:, 1:2] * dx * dy
        G = torch.exp(power)
        alpha = torch.clamp(opacity[g][:, None] * G, max=0.99)
        act = act & (power <= 0) & (alpha >= 1.0 / 255.0)
        af = act.float()
        Tr = torch.where(act, Tr / (1 - alpha), Tr)
        dch = alpha * Tr
        c = feat[g][:, None, :].expand_as(dL_dpix)
        accum = torch.where(act[:, :, None], last_alpha[:, :, None] * last_color
                            + (1 - last_alpha[:, :, None]) * accum, accum)
        last_color = torch.where(act[:, :, None], c, last_color)
        dL_dalpha = ((c - accum) * dL_dpix).sum(-1)
        g_col.index_add_(0, g, ((dch * af)[:, :, None] * dL_dpix).sum(1))
        dL_dalpha = dL_dalpha * Tr
        last_alpha = torch.where(act, alpha, last_alpha)
        dL_dalpha = dL_dalpha + (-final_T / (1 - alpha)) * bg_dot
        dL_dG = opacity[g][:, None] * dL_dalpha * af
        gdx, gdy = G * dx, G * dy
        dG_ddx = -gdx * co[:, 0:1] - gdy * co[:, 1:2]
        dG_ddy = -gdy * co[:, 2:3] - gdx * co[:, 1:2]
        gm = torch.stack([(dL_dG * dG_ddx).sum(1) * (0.5 * W), (dL_dG * dG_ddy).sum(1) * (0.5 * H),
                          torch.zeros_like(g, dtype=torch.float32)], 1)
        g_mean.index_add_(0, g, gm)
        gc = torch.stack([(-0.5 * gdx * dx * dL_dG).sum(1), (-0.5 * gdx * dy * dL_dG).sum(1),
                          torch.zeros(g.shape[0]), (-0.5 * gdy * dy * dL_dG).sum(1)], 1)
        g_conic.view(P, 4).index_add_(0, g, gc)
        g_op.index_add_(0, g, (G * dL_dalpha * af).sum(1)[:, None])
    return dict(dL_dmean2D=g_mean, dL_dconic=g_conic, dL_dopacity=g_op, dL_dcolors=g_col)


def preprocess_bwd(pre, leaves, dL_dmean2D, dL_dconic, dL_dcolors):
    """computeCov2DCUDA + preprocessCUDA backward by autograd through `preprocess`
    (leaves: the tensors it was called with, requiring grad)."""
    vis = (pre["radii"] > 0).float()[:, None]
    g_ndc = dL_dmean2D[:, 0:2] * vis
    g_con = torch.stack([dL_dconic[:, 0, 0], 2.0 * dL_dconic[:, 0, 1], dL_dconic[:, 1, 1]], 1) * vis
    outs, gouts = [pre["ndc"], pre["conic"]], [g_ndc, g_con]
    if pre["rgb"].requires_grad:
        outs.append(pre["rgb"])
        gouts.append(dL_dcolors * vis)
    return torch.autograd.grad(outs, leaves, gouts, allow_unused=True)


def rasterize(means3D, scales, rotations, opacities, shs, deg, viewmatrix, projmatrix, campos, W, H, tanfovx,
              tanfovy, bg, colors=None, tiles=None, tile_batch=None):
    """Forward of the given tiles (all when None): returns (pre, point_list, ranges, out)
    with out = (color, final_T, n_contrib, inside, tiles)."""
    with torch.no_grad():
        pre = preprocess(means3D, scales, rotations, opacities, shs, deg, viewmatrix, projmatrix, campos, W, H,
                         tanfovx, tanfovy, colors=colors)
        pl, ranges = binning(pre, W, H)
    T = ranges.shape[0]
    tiles = torch.arange(T) if tiles is None else torch.as_tensor(tiles, dtype=torch.int64)
    out = render_fwd(tiles, ranges, pl, pre["xy"], pre["conic"].detach(), pre["opacity"], pre["rgb"].detach(), bg,
                     W, H)
    return pre, pl, ranges, out + (tiles,)


def to_image(vals, tiles, W, H, C=3):
    """[nt,256,C] tile-major values -> [C,H,W] image (pixels of other tiles 0)."""
    gx = (W + BLOCK - 1) // BLOCK
    img = torch.zeros(C, (H + BLOCK - 1) // BLOCK * BLOCK, gx * BLOCK)
    v = vals.reshape(-1, BLOCK, BLOCK, C)
    for i, t in enumerate(tiles.tolist()):
        bx, by = t % gx, t // gx
        img[:, by * BLOCK:(by + 1) * BLOCK, bx * BLOCK:(bx + 1) * BLOCK] = v[i].permute(2, 0, 1)
    return img[:, :H, :W]


def from_image(img, tiles, W, H):
    """[C,H,W] image -> [nt,256,C] for the given tiles (outside pixels 0)."""
    gx = (W + BLOCK - 1) // BLOCK
    Hp, Wp = (H + BLOCK - 1) // BLOCK * BLOCK, gx * BLOCK
    pad = torch.zeros(img.shape[0], Hp, Wp)
    pad[:, :H, :W] = img
    t = tiles
    bx, by = t % gx, t // gx
    ly = torch.arange(BLOCK)
    rows = (by[:, None] * BLOCK + ly[None, :])  # [nt,16]
    cols = (bx[:, None] * BLOCK + ly[None, :])
    v = pad[:, rows[:, :, None], cols[:, None, :]]  # [C,nt,16,16]
    return v.permute(1, 2, 3, 0).reshape(t.numel(), BLOCK * BLOCK, img.shape[0])


def host_threads():
    """The cores this process may use: the affinity mask, capped by OMP_NUM_THREADS when set
    (on the GPU box os.cpu_count() reports the whole machine, not this job's share)."""
    import os
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)


def sample_tiles(T, n, seed=2):
    g = torch.Generator().manual_seed(seed)
    return torch.randperm(T, generator=g)[:min(n, T)].sort().values

