"""The backward tile pass's dispatch order, bit-exact against a numpy restatement.

The forward tile pass leaves, per 16x16 tile, the backward's cost estimate (the sum of its four
8x8 quadrants' largest n_contrib) and its per-tile-row sums; the backward's order launch
(k_tile_order, gsr_order.hpp) cuts the tiles into 8 contiguous XCD bands holding equal shares of
cost' = estimate + a floor (balanced_band), and orders each band by cost bucket, heaviest first.
Integer work, so every array is compared exactly: the estimate against n_contrib, the row sums,
the band bounds, and each band's order (a permutation of its range, buckets descending, within
the launch's grid bound).  Frames with more than 512 tile rows or tiles per row take equal bands."""
import numpy as np
import pytest
import torch

from helpers import make_case
from test_gpu_rasterizer import _dgr, _view, mutate, run_gpu

pytestmark = pytest.mark.gpu

BUCKET_FRAC = 3  # gsr_order.hpp GSR_BUCKET_BITS


def cost_bucket(c):
    """gsr_order.hpp cost_bucket: the bit length of c and its next BUCKET_FRAC bits."""
    c = int(c)
    if c == 0:
        return 0
    L = c.bit_length()
    fm = (1 << BUCKET_FRAC) - 1
    f = (c >> (L - 1 - BUCKET_FRAC)) & fm if L > BUCKET_FRAC else (c << (BUCKET_FRAC + 1 - L)) & fm
    return (L << BUCKET_FRAC) + f


def equal_bounds(ntile):
    """gsr_tile.hpp band_of: the first ntile % 8 bands hold one tile more."""
    q, r = divmod(ntile, 8)
    return [b * (q + 1) if b < r else r * (q + 1) + (b - r) * q for b in range(8)] + [ntile]


def balanced_bounds(cost, gx, gy):
    """gsr_order.hpp balanced_band, restated over the whole frame."""
    ntile = gx * gy
    total = int(cost.astype(np.uint64).sum())
    if gy > 512 or gx > 512 or total == 0:
        return equal_bounds(ntile)
    add = -(-total // (2 * ntile))  # half the mean tile cost, rounded up
    tp = total + add * ntile
    incl = np.cumsum(cost.astype(np.int64) + add)
    return [0] + [int(np.searchsorted(incl, k * tp // 8, side="left")) + 1 for k in range(1, 8)] + [ntile]


def quadrant_maxima_sum(n_contrib, W, H, gx, gy):
    nc = np.zeros((gy * 16, gx * 16), np.int64)
    nc[:H, :W] = n_contrib.reshape(H, W)
    q = nc.reshape(gy, 2, 8, gx, 2, 8).max(axis=(2, 5))  # [gy, 2, gx, 2]
    return q.sum(axis=(1, 3)).reshape(-1)


CASES = [
    dict(name="uniform_640x360", P=20000, W=640, H=360),
    dict(name="opaque_400x300", P=8000, W=400, H=300, mutate="opaque"),
    dict(name="clustered_512x512", P=12000, W=512, H=512, mutate="cluster"),
    dict(name="wide_strip_fallback", P=3000, W=8320, H=40),
]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_backward_order(case):
    _, _C, _lib = _dgr()
    W, H = case["W"], case["H"]
    cam, gs = make_case(P=case["P"], W=W, H=H, sh_degree=0)
    how = case.get("mutate")
    if how == "cluster":  # a quarter of the cloud squeezed onto a small patch: skewed tile costs
        gs = {k: v.clone() for k, v in gs.items()}
        n = gs["means3D"].shape[0] // 4
        gs["means3D"][:n, :2] = gs["means3D"][:n, :2] * 0.05 + 0.1 * gs["means3D"][:n, 2:3]
    else:
        gs = mutate(gs, how)
    st = run_gpu(cam, gs, mode="colors")
    dout = torch.randn(3, H, W, generator=torch.Generator().manual_seed(3)).cuda()
    _C.rasterize_gaussians_backward(
        st["bg"], st["means"], st["radii"], st["colors"], st["scales"], st["rots"], 1.0, st["cov3"], st["vm"],
        st["pm"], cam.tanfovx, cam.tanfovy, dout, st["sh"], 0, st["cp"], st["geom"], st["R"], st["binb"], st["img"])
    torch.cuda.synchronize()
    gx, gy = (W + 15) // 16, (H + 15) // 16
    ntile = gx * gy
    L = _lib.layout(case["P"], st["R"], W, H)
    img = st["img"]
    cost = _view(img, L.img_tile_cost, ntile, torch.int32).cpu().numpy().view(np.uint32).astype(np.int64)
    rows = _view(img, L.img_row_cost, gy, torch.int32).cpu().numpy().view(np.uint32).astype(np.int64)
    order = _view(img, L.img_order_bwd, ntile, torch.int32).cpu().numpy().view(np.uint32).astype(np.int64)
    table = _view(img, L.img_nheavy, 32, torch.int32).cpu().numpy().view(np.uint32).astype(np.int64)

    # the estimate (the forward's (survivor, quadrant) evaluations, GSR_EVAL_COST: positive exactly on
    # the tiles with a contributor, at least one evaluation per contributing quadrant) and its row sums
    qmax = quadrant_maxima_sum(st["n_contrib"], W, H, gx, gy)
    np.testing.assert_array_equal(cost > 0, qmax > 0)
    np.testing.assert_array_equal(rows, cost.reshape(gy, gx).sum(axis=1))
    assert cost.sum() > 0

    # the bands: bounds, partition, grid bound (tile_pass_blocks_bal), order
    bounds = [int(x) for x in table[16:25]]
    assert bounds == balanced_bounds(cost, gx, gy), (bounds, balanced_bounds(cost, gx, gy))
    if case["name"].endswith("fallback"):
        assert bounds == equal_bounds(ntile)
    if how == "cluster":  # skewed costs: the bands really move
        assert bounds != equal_bounds(ntile)
    cap = 3 * ((ntile + 7) // 8) + 2
    for b in range(8):
        lo, hi = bounds[b], bounds[b + 1]
        assert 0 <= hi - lo <= cap
        seg = order[lo:hi]
        np.testing.assert_array_equal(np.sort(seg), np.arange(lo, hi))
        bk = np.array([cost_bucket(c) for c in cost[seg]])
        assert np.all(np.diff(bk) <= 0), f"band {b} not heaviest-first"
    # balanced (not the fallback): every band's cost' share is within one tile's cost' of 1/8
    if not case["name"].endswith("fallback"):
        total = int(cost.sum())
        add = -(-total // (2 * ntile))
        share = np.array([(cost[bounds[b]:bounds[b + 1]] + add).sum() for b in range(8)])
        assert share.max() - share.min() <= 2 * int(cost.max() + add)
