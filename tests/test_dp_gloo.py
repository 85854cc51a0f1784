"""World-size-2 gloo tests of the view-parallel DP path (gsr/dp.py) on the CPU.

The reduced gradients and densification statistics of 2 ranks x 2 views must equal the
single-process accumulation over the same 4 views (the reference's sequential loop), to float
summation-order tolerance; max_radii2D is exact."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import dp_worker


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_views_partition():
    from gsr import dp
    for world in (1, 2, 3, 8):
        got = sorted(v for r in range(world) for v in dp.shard_views(10, r, world))
        assert got == list(range(10))
    with pytest.raises(ValueError):
        dp.shard_views(4, 2, 2)


def test_grad_bucket_roundtrip_single_process():
    from gsr import dp
    ts = [torch.randn(5, 3), torch.randn(5, 1), torch.randn(7)]
    b = dp.GradBucket(ts)
    b.pack(ts)
    assert b.flat.numel() == 15 + 5 + 7
    outs = [torch.zeros_like(t) for t in ts]
    b.unpack(outs)
    for a, o in zip(ts, outs):
        assert torch.equal(a, o)
    with pytest.raises(ValueError):
        b.pack([torch.randn(4, 3), ts[1], ts[2]])


def test_view_parallel_step_matches_sequential(tmp_path):
    out = str(tmp_path / "rank0.npz")
    mp.spawn(dp_worker.run, args=(2, free_port(), out), nprocs=2, join=True)
    got = np.load(out, allow_pickle=False)
    ref_grads, ref_stats = dp_worker.local_step(0, 1, views=[0, 1, 2, 3])
    for k, t in zip(dp_worker.GRAD_KEYS, ref_grads):
        r = t.numpy()
        err = np.linalg.norm(got[k] - r) / max(np.linalg.norm(r), 1e-30)
        assert err <= 1e-6, (k, err)
    assert np.array_equal(got["denom"], ref_stats["denom"].numpy())
    assert np.array_equal(got["max_radii2D"], ref_stats["max_radii2D"].numpy())
    np.testing.assert_allclose(got["xyz_gradient_accum"], ref_stats["xyz_gradient_accum"].numpy(), rtol=1e-6,
                               atol=1e-9)
    assert ref_stats["denom"].max().item() >= 2  # views overlap: the sums are non-trivial


def test_multi_step_stats_and_rank_consistent_densify(tmp_path):
    """the running statistics must equal the sequential accumulation after
    SEVERAL steps (each step's deltas are reduced, not the running totals).  Then one
    densify_and_prune (gaussian_model.py:610-625) on both ranks from the shared generator:
    P, parameters, Adam moments, step count and sky flags bit-identical on the ranks."""
    out = str(tmp_path / "densify.npz")
    mp.spawn(dp_worker.run_densify, args=(2, free_port(), out), nprocs=2, join=True)
    got = np.load(out, allow_pickle=False)
    ref = dp_worker.stats_run(0, 1)
    assert np.array_equal(got["denom"], ref["denom"].numpy())
    assert float(ref["denom"].max()) > dp_worker.N_STEPS  # several views per step, several steps
    assert np.array_equal(got["max_radii2D"], ref["max_radii2D"].numpy())
    np.testing.assert_allclose(got["xyz_gradient_accum"], ref["xyz_gradient_accum"].numpy(), rtol=1e-6, atol=1e-7)
    same = got["identical"]  # parameters, both moments, sky flags, (P, t): byte-equal on both ranks
    assert same.shape == (5,) and same.all(), same
    P0 = dp_worker.small_scene().P
    assert int(got["P"]) != P0  # the surgery did something
    assert int(got["t"]) == 7


def test_densify_matches_sequential_with_same_seed():
    """Single process: the same views' statistics and the same seed give the same scene as
    the ranks (clone + split + prune all exercised)."""
    a = dp_worker.densify_run(0, 1, seed=11)
    b = dp_worker.densify_run(0, 1, seed=11)
    assert a.P == b.P and torch.equal(a.fp.flat, b.fp.flat) and torch.equal(a.fp.exp_avg_sq, b.fp.exp_avg_sq)
    base = dp_worker.small_scene()
    assert a.P != base.P
    # the Adam moments of appended rows are zero; kept rows carry theirs
    assert a.fp.exp_avg.abs().sum() > 0


def test_replicas_identical_sees_one_bit(tmp_path):
    """The replica check compares bytes: -0.0 against +0.0 and a shape difference are caught."""
    out = str(tmp_path / "flags.npy")
    mp.spawn(dp_worker.run_identical_probe, args=(2, free_port(), out), nprocs=2, join=True)
    assert np.load(out).tolist() == [False, True, False]


def test_iteration_exchange_is_one_pipelined_collective(tmp_path):
    """gsr.dp.finish_step (train_step's tail) issues ONE logical
    exchange per iteration at world size 2 -- the flat gradient's SUM all-reduce, carrying the
    step's densification sums in its tail below densify_until_iter and the gradient alone past
    it -- sent as EX_CHUNKS consecutive slices that together cover the bucket exactly once, and
    hands the optimizer every gradient element exactly once, slice by slice in order (the
    pipelined Adam); the result equals the sequential accumulation over both ranks' views:
    gradient bit-exact (two-rank sums commute, and a SUM is elementwise, so slicing changes no
    bit), denom and max_radii2D exact (the rank-local maxima MAX-reduced once, as densification
    does), the norm accumulator to float order; the sums stop at iteration 15000 (train.py:143)
    while max_radii2D keeps updating (train.py:130)."""
    out = str(tmp_path / "exchange.npz")
    mp.spawn(dp_worker.run_exchange, args=(2, free_port(), out), nprocs=2, join=True)
    got = np.load(out, allow_pickle=False)
    ref, ref_counts, ref_opt, _ = dp_worker.exchange_run(0, 1)
    K = dp_worker.EX_CHUNKS
    assert got["counts"].tolist() == [[K, K]] * len(dp_worker.EX_ITERS), got["counts"]
    assert [c[0] for c in ref_counts] == [0] * len(dp_worker.EX_ITERS)
    n, P = ref.fp.n, ref.P
    # the slices carry the whole bucket: gradient + sums below 15000, the gradient alone after
    want = [n + 2 * P if it < 15000 else n for it in dp_worker.EX_ITERS]
    assert got["sizes"].tolist() == want and got["nsizes"].tolist() == [K] * len(want)
    # the optimizer sees [0, n) once per iteration, in ascending contiguous ranges
    per = got["opt_per_it"].tolist()
    rs = got["opt"].tolist()
    i = 0
    for k in per:
        its = rs[i:i + k]
        i += k
        assert its[0][0] == 0 and its[-1][1] == n and all(a[1] == b[0] for a, b in zip(its, its[1:]))
        assert all(lo % 4 == 0 for lo, _ in its)
    assert all(r == [[0, n]] for r in [[list(x) for x in it] for it in ref_opt])
    assert int(got["tail"]) == 2 * ref.P
    assert np.array_equal(got["grad"], ref.fp.grad.numpy())
    assert np.array_equal(got["denom"], ref.stats["denom"].numpy())
    assert np.array_equal(got["max_radii2D"], ref.stats["max_radii2D"].numpy())
    np.testing.assert_allclose(got["xyz_gradient_accum"], ref.stats["xyz_gradient_accum"].numpy(), rtol=1e-6,
                               atol=1e-7)
    # two iterations below densify_until_iter (14998, 14999) count; 15000 and 15001 do not
    on = sum(1 for it in dp_worker.EX_ITERS if it < 15000)
    assert float(ref.stats["denom"].max()) <= on * 2 * dp_worker.VIEWS_PER_RANK
    assert float(ref.stats["denom"].max()) >= on
    # max_radii2D did take the last iterations' views
    _, r_last = dp_worker.view_stats(dp_worker.EX_ITERS[-1], 0, ref.P)
    assert (ref.stats["max_radii2D"] >= r_last.float()).all()


def test_reference_loop_exchange(tmp_path):
    """gsr.dp.ReferenceExchange (INTEGRATION.md's recipe for the reference's own train.py loop):
    one exchange per iteration (2 pipelined slices here), gradients summed over the ranks bit
    for bit, the statistics deltas folded in while they are on, and max_radii2D equal after the
    one MAX-reduce densification makes."""
    out = str(tmp_path / "refex.npz")
    mp.spawn(dp_worker.run_refex, args=(2, free_port(), out), nprocs=2, join=True)
    got = np.load(out, allow_pickle=False)
    g, grads, issued = dp_worker.refex_run(0, 1)
    assert got["issued"].tolist() == [2, 2] and issued == [0, 0]
    assert np.array_equal(got["xyz0"], grads[0][0].numpy())
    assert np.array_equal(got["alb1"], grads[1][1].numpy())
    assert np.array_equal(got["denom"], g.denom.numpy())
    assert np.array_equal(got["max_radii2D"], g.max_radii2D.numpy())
    np.testing.assert_allclose(got["accum"], g.xyz_gradient_accum.numpy(), rtol=1e-6, atol=1e-7)


def test_reference_exchange_follows_densify(tmp_path):
    """ReferenceExchange(optimizer=...) across a densify_and_prune-style resize: the
    replaced, larger Gaussian Parameter and the resized statistics are exchanged in the next
    iteration without a rebuild, an MLP weight that only one rank's views reach and the sky radius
    stay identical on every rank, everything equals the one-process run over both ranks' views,
    and a fixed-list exchange built for the old size refuses the resized statistics."""
    out = str(tmp_path / "refex_resize.npz")
    mp.spawn(dp_worker.run_refex_resize, args=(2, free_port(), out), nprocs=2, join=True)
    got = np.load(out, allow_pickle=False)
    assert got["same"].all(), got["same"]
    want = dp_worker.refex_resize_run(0, 1)
    assert want["xyz"].shape == (260, 3) and bool(got["refused"]) and bool(want["refused"])
    for k in ("xyz", "mlp", "sky", "accum", "denom"):
        np.testing.assert_allclose(got[k], want[k], rtol=1e-6, atol=1e-7, err_msg=k)


def test_exchange_chunks_cover_aligned():
    """gsr.dp.exchange_chunks: contiguous ascending slices covering [0, n) exactly once, every
    start a multiple of 4 floats (the ranged Adam's float4 rows), at most `chunks` of them,
    none below the size floor unless the bucket itself is smaller."""
    from gsr import dp
    for n, k, floor in ((23_316_836 + 3_000_000, 4, 1 << 20), (10, 4, 1 << 20), (1001, 3, 1), (4096, 8, 100),
                        (7, 8, 1), (0, 4, 1)):
        r = dp.exchange_chunks(n, k, floor)
        if n == 0:
            assert r == [(0, 0)]
            continue
        assert r[0][0] == 0 and r[-1][1] == n and all(a[1] == b[0] for a, b in zip(r, r[1:]))
        assert all(lo % 4 == 0 and hi > lo for lo, hi in r)
        assert 1 <= len(r) <= k
        if n >= k * floor:
            assert len(r) == k
