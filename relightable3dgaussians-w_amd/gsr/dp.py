"""View-parallel data parallelism for the rasterizer path.

The reference trains on one camera per iteration (train.py:95-160): render -> loss ->
backward -> densification statistics -> Adam.  The only part of that loop that touches
every Gaussian on every view is the per-Gaussian gradient and the densification statistics,
so the MI355X design shards *views* over ranks (one process per GPU, weak scaling) and adds
exactly one exchange step per iteration:

  * the per-Gaussian gradients of all parameters are flattened into ONE contiguous bucket
    and summed with a single all-reduce (RCCL over xGMI on the GPU box, gloo in the CPU
    tests).  Summing N single-view gradients is what the reference computes by accumulating
    N iterations of batch 1 before a step.  One large bucket beats many small ones on xGMI:
    at cfg2 the bucket is 1.5M x 59 floats = 354 MB, which amortises ring latency.
  * the densification statistics: ``xyz_gradient_accum`` and ``denom``
    (gaussian_model.py:627-629) are SUMmed, ``max_radii2D`` (train.py:130) is MAXed.  Each
    rank accumulates ONE STEP's views into zeroed per-step buffers (StepStats); only those
    deltas are reduced and then folded into the running statistics, so after any number of
    steps the running statistics equal the sequential reference's over the same views
    (reducing the running totals instead would re-multiply every earlier step by the world
    size).
  * densification (gaussian_model.py:610-625) stays rank-consistent: the statistics and
    parameters are identical on every rank by construction, and the only random draw (the
    split's torch.normal, :560) comes from a generator seeded with a value broadcast from
    rank 0 (``shared_generator`` / ``consistent_rng``), so every rank clones, splits and
    prunes the same Gaussians and draws the same samples.

No collective touches the rasterizer itself: every rank calls the same libgsr.so on its own
view.  The helpers take any process group, so the gloo world_size-2 tests in
tests/test_dp_gloo.py exercise the same code the nccl bench path runs.
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist


def shard_views(n_views: int, rank: int, world: int) -> List[int]:
    """Round-robin view assignment: rank r renders views r, r+world, ... (disjoint, covering)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    return list(range(rank, n_views, world))


class GradBucket:
    """One flat buffer holding several gradient tensors back to back.

    ``pack`` copies the tensors in, ``all_reduce`` runs one collective over the whole buffer,
    and ``unpack`` copies the reduced values back into the original tensors, in place.  The
    buffer is allocated once and reused, so a training step does not allocate.
    """

    def __init__(self, like: Sequence[torch.Tensor]):
        if not like:
            raise ValueError("GradBucket needs at least one tensor")
        dt, dev = like[0].dtype, like[0].device
        for t in like:
            if t.dtype != dt or t.device != dev:
                raise ValueError("GradBucket tensors must share dtype and device")
        self.shapes = [tuple(t.shape) for t in like]
        self.sizes = [t.numel() for t in like]
        self.flat = torch.empty(sum(self.sizes), dtype=dt, device=dev)

    def views(self) -> List[torch.Tensor]:
        out, o = [], 0
        for n, shp in zip(self.sizes, self.shapes):
            out.append(self.flat[o:o + n].view(shp))
            o += n
        return out

    def pack(self, tensors: Sequence[torch.Tensor]) -> None:
        if [tuple(t.shape) for t in tensors] != self.shapes:
            raise ValueError("GradBucket.pack: shapes differ from the bucket layout")
        for v, t in zip(self.views(), tensors):
            v.copy_(t)

    def unpack(self, tensors: Sequence[torch.Tensor]) -> None:
        for v, t in zip(self.views(), tensors):
            t.copy_(v)

    def all_reduce(self, group=None, average: bool = False) -> None:
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
        if average:
            self.flat.div_(dist.get_world_size(group))


def all_reduce_grads(tensors: Sequence[torch.Tensor], bucket: Optional[GradBucket] = None, group=None,
                     average: bool = False) -> GradBucket:
    """Sum (or average) ``tensors`` over the group with a single collective, in place."""
    if bucket is None:
        bucket = GradBucket(tensors)
    bucket.pack(tensors)
    bucket.all_reduce(group=group, average=average)
    bucket.unpack(tensors)
    return bucket


def reduce_densification_stats(xyz_gradient_accum: torch.Tensor, denom: torch.Tensor, max_radii2D: torch.Tensor,
                               group=None) -> None:
    """In place: SUM the gradient-norm accumulator and the view counter, MAX the screen radii.

    Mirrors gaussian_model.py:627-629 (accum += ||dL/dmean2D[:, :2]||, denom += 1 on the
    visibility filter) and train.py:130 (max_radii2D = max(max_radii2D, radii)) across ranks.
    The two sums travel in one buffer.
    """
    sums = torch.cat([xyz_gradient_accum.reshape(-1), denom.reshape(-1)])
    dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)
    n = xyz_gradient_accum.numel()
    xyz_gradient_accum.copy_(sums[:n].view_as(xyz_gradient_accum))
    denom.copy_(sums[n:].view_as(denom))
    dist.all_reduce(max_radii2D, op=dist.ReduceOp.MAX, group=group)


def accumulate_view_stats(stats: Dict[str, torch.Tensor], mean2D_grad: torch.Tensor, radii: torch.Tensor) -> None:
    """Per-rank, per-view densification update (train.py:130, gaussian_model.py:627-629)."""
    # dense masked updates (no boolean indexing: that is a nonzero + host sync per array)
    vis = radii > 0
    mr = stats["max_radii2D"]
    torch.where(vis, torch.maximum(mr, radii.to(mr.dtype)), mr, out=mr)
    v1 = vis[:, None]
    stats["xyz_gradient_accum"].add_(torch.where(v1, torch.norm(mean2D_grad[:, :2], dim=-1, keepdim=True), 0.0))
    stats["denom"].add_(v1.to(stats["denom"].dtype))


class StepStats:
    """One step's densification deltas on this rank (train.py:130, gaussian_model.py:627-629).

    ``zero()`` at the start of a step, ``add_view`` per rendered view, ``commit`` once per
    step: the deltas are reduced across ranks (SUM for the norm accumulator and the view
    counter, MAX for the radii) and then added to / maxed into the running statistics.
    Preallocated; a step allocates nothing."""

    def __init__(self, P: int, device):
        self.d = {"xyz_gradient_accum": torch.zeros(P, 1, device=device), "denom": torch.zeros(P, 1, device=device),
                  "max_radii2D": torch.zeros(P, device=device)}

    @classmethod
    def view_of(cls, stats: Dict[str, torch.Tensor]) -> "StepStats":
        """A StepStats over existing statistics tensors (add_views then updates them in place)."""
        obj = cls.__new__(cls)
        obj.d = stats
        return obj

    def zero(self) -> None:
        for t in self.d.values():
            t.zero_()

    def add_view(self, mean2D_grad: torch.Tensor, radii: torch.Tensor) -> None:
        accumulate_view_stats(self.d, mean2D_grad, radii)

    def add_views(self, mean2D_grads, radii) -> None:
        """add_view over the views in order; on GPU tensors one HIP pass for up to 8 views
        (gsr_densify_stats) instead of ~8 elementwise kernels per view."""
        if not mean2D_grads[0].is_cuda:
            for g, r in zip(mean2D_grads, radii):
                self.add_view(g, r)
            return
        from . import _lib
        d = self.d
        P = d["denom"].shape[0]
        for i in range(0, len(radii), 8):
            gs = [g.contiguous() for g in mean2D_grads[i:i + 8]]
            rs = [r.contiguous() for r in radii[i:i + 8]]
            _lib.check(_lib.lib().gsr_densify_stats(P, len(rs), _lib.ptr_array(gs), _lib.ptr_array(rs),
                                                    d["xyz_gradient_accum"].data_ptr(), d["denom"].data_ptr(),
                                                    d["max_radii2D"].data_ptr(), _lib.stream_of(gs[0].device)),
                       "gsr_densify_stats")

    def commit(self, running: Dict[str, torch.Tensor], group=None, world: int = 1) -> None:
        d = self.d
        if world > 1:
            reduce_densification_stats(d["xyz_gradient_accum"], d["denom"], d["max_radii2D"], group=group)
        running["xyz_gradient_accum"].add_(d["xyz_gradient_accum"])
        running["denom"].add_(d["denom"])
        torch.maximum(running["max_radii2D"], d["max_radii2D"], out=running["max_radii2D"])


# ---- the training iteration's exchange (gsr.train.train_step) ------------------------------

DENSIFY_UNTIL_ITER = 15000  # configs/optimizer/optimization_params.yaml:16 densify_until_iter


def add_views(accum: Optional[torch.Tensor], denom: Optional[torch.Tensor], max_radii: torch.Tensor,
              mean2D_grads, radii) -> None:
    """The views' densification updates in view order (train.py:130, gaussian_model.py:627-629):
    max_radii = max(max_radii, radii) on the visible Gaussians and, unless accum / denom are
    None, accum += ||dL/dmean2D[:, :2]||, denom += 1.  On GPU tensors one HIP pass per 8 views
    (gsr_densify_stats)."""
    if not radii[0].is_cuda:
        for g, r in zip(mean2D_grads, radii):
            vis = r > 0
            torch.where(vis, torch.maximum(max_radii, r.to(max_radii.dtype)), max_radii, out=max_radii)
            if accum is not None:
                v1 = vis[:, None]
                accum.add_(torch.where(v1, torch.norm(g[:, :2], dim=-1, keepdim=True), 0.0))
                denom.add_(v1.to(denom.dtype))
        return
    from . import _lib
    P = max_radii.shape[0]
    ptr = lambda t: None if t is None else t.data_ptr()
    for i in range(0, len(radii), 8):
        rs = [r.contiguous() for r in radii[i:i + 8]]
        gs = [g.contiguous() for g in mean2D_grads[i:i + 8]] if accum is not None else None
        _lib.check(_lib.lib().gsr_densify_stats(P, len(rs), None if gs is None else _lib.ptr_array(gs),
                                                _lib.ptr_array(rs), ptr(accum), ptr(denom), max_radii.data_ptr(),
                                                _lib.stream_of(rs[0].device)), "gsr_densify_stats")


def step_sums(fp, P: int):
    """This step's densification sums (xyz_gradient_accum and denom deltas, [P,1] each) as views
    of the flat gradient's tail, zeroed with it by FlatParams.zero_grad."""
    if fp.tail < 2 * P:
        raise RuntimeError(f"the flat gradient's tail holds {fp.tail} floats, the step's sums need {2 * P}")
    t = fp.grad_tail
    return t[:P].view(P, 1), t[P:2 * P].view(P, 1)


def sync_max_radii(stats: Dict[str, torch.Tensor], group=None) -> None:
    """max_radii2D stays rank-local between densifications: MAX is associative and only
    densify_and_prune reads it (gaussian_model.py:620), so the ranks' running maxima are
    MAX-reduced once, right before it does (gsr.densify.densify_and_prune)."""
    dist.all_reduce(stats["max_radii2D"], op=dist.ReduceOp.MAX, group=group)


def synced_stats(scene, group=None) -> Dict[str, torch.Tensor]:
    """scene.stats with every field rank-consistent: the one call any reader other than
    densification (a checkpoint, a statistics export, another pruning path) must make before it
    reads them at N > 1.  While ``scene.max_radii_local`` is set, max_radii2D holds this rank's
    views only (finish_step leaves it rank-local); this MAX-reduces it (a collective: every rank
    must call it) and clears the mark.  The sums are always consistent (they ride in the
    iteration's exchange)."""
    if getattr(scene, "max_radii_local", False):
        if dist.is_available() and dist.is_initialized():
            sync_max_radii(scene.stats, group)
        scene.max_radii_local = False
    return scene.stats


EXCHANGE_CHUNKS = 4  # the data-parallel step's all-reduce, in this many pipelined chunks
EXCHANGE_MIN_CHUNK = 1 << 20  # floats: smaller buckets go out whole


def exchange_chunks(n: int, chunks: int = EXCHANGE_CHUNKS, min_chunk: int = EXCHANGE_MIN_CHUNK):
    """[lo, hi) ranges cutting a bucket of n floats into at most ``chunks`` pieces of at least
    ``min_chunk`` floats (each start a multiple of 4: the Adam kernel's float4 rows)."""
    k = max(1, min(int(chunks), n // max(1, int(min_chunk))))
    step = -(-n // k)
    step = (step + 3) & ~3
    out, lo = [], 0
    while lo < n:
        out.append((lo, min(n, lo + step)))
        lo += step
    return out or [(0, 0)]


def finish_step(scene, mean2D_grads, radii, iteration: int, world: int = 1, group=None, on_chunk=None,
                chunks: int = None, min_chunk: int = None) -> int:
    """The tail of gsr.train.train_step after the views' backward: the densification
    statistics, the iteration's exchange and (``on_chunk``) the optimizer step.  Returns the
    number of collectives it issued.

    * train.py:130 updates max_radii2D every iteration; train.py:143-144 adds the gradient-norm
      sums only while iteration < densify_until_iter.
    * One rank: straight into the running statistics; on_chunk(0, n) updates every parameter.
    * N ranks: one SUM all-reduce of the flat bucket per iteration -- the gradient, and while
      the statistics are on, the step's sums in the bucket's tail (step_sums: [gradient | accum
      deltas | denom deltas]), folded into the running statistics after; past
      densify_until_iter the bucket is the gradient alone.  The bucket goes out as ``chunks``
      (default EXCHANGE_CHUNKS) consecutive slices, all issued at once (asynchronously, in
      order, on the collective stream); on_chunk(lo, hi) runs the optimizer over the gradient
      part of slice i as soon as slice i has landed (work.wait orders the current stream after
      it), so the update of slice i overlaps the exchange of slices i + 1... .  A SUM is
      elementwise, so the slices reduce exactly as the whole bucket would.  max_radii2D is
      updated rank-locally (sync_max_radii reduces it when densification needs it);
      ``scene.max_radii_local`` marks it."""
    st = scene.stats
    stats_on = iteration < DENSIFY_UNTIL_ITER
    fp = scene.fp
    if world > 1:
        acc, den = step_sums(fp, scene.P) if stats_on else (None, None)
        scene.max_radii_local = True
    else:
        acc, den = (st["xyz_gradient_accum"], st["denom"]) if stats_on else (None, None)
    add_views(acc, den, st["max_radii2D"], mean2D_grads, radii)
    if world <= 1:
        if on_chunk is not None:
            on_chunk(0, fp.n)
        return 0
    bucket = fp.bucket(stats_on)
    ranges = exchange_chunks(bucket.numel(), EXCHANGE_CHUNKS if chunks is None else chunks,
                             EXCHANGE_MIN_CHUNK if min_chunk is None else min_chunk)
    works = [dist.all_reduce(bucket[lo:hi], op=dist.ReduceOp.SUM, group=group, async_op=True) for lo, hi in ranges]
    for (lo, hi), w in zip(ranges, works):
        w.wait()
        if on_chunk is not None and lo < fp.n:
            on_chunk(lo, min(hi, fp.n))
    if stats_on:
        st["xyz_gradient_accum"].add_(acc)
        st["denom"].add_(den)
    return len(ranges)


class ReferenceExchange:
    """The reference's own training loop (train.py:116-163, GaussianModel tensors) under view
    parallelism with the same single exchange as finish_step: one flat bucket holds every
    exchanged parameter's gradient and, while densification statistics are on
    (train.py:143: iteration < densify_until_iter), this iteration's norm-accumulator and view
    count deltas; one SUM all-reduce (in pipelined slices) per iteration moves both.
    max_radii2D stays rank-local (train.py:130 MAX is associative): call
    ``sync_max_radii({"max_radii2D": g.max_radii2D})`` right before densify_and_prune, or
    ``synced`` before any other reader.

        ex = dp.ReferenceExchange(optimizer=g.optimizer)
        ...loss.backward()
        ex.add_views([viewspace_point_tensor.grad], [radii], g.max_radii2D, stats_on)
        ex.exchange(g, stats_on, world=dist.get_world_size())   # grads summed in place

    With ``optimizer`` (the recommended form) the exchanged parameters are, on every call, every
    tensor with requires_grad in its param_groups -- the Gaussians' attributes, the sky radius
    (gaussian_model.py:272) and, in the relightable model, the MLP and appearance embeddings
    (relit3DGW_model.py:144-145) -- so nothing drifts apart across ranks, and the
    densify_and_prune that replaces the Parameters and resizes the statistics
    (gaussian_model.py:471-542) needs no rebuild: the bucket is re-laid out for the new sizes.
    With a fixed ``params`` list and ``P`` the exchange checks on every call that the statistics
    still hold P rows and that every listed tensor is still the size it was, and raises
    otherwise (rebuild it after densify_and_prune)."""

    def __init__(self, params: Optional[Sequence[torch.Tensor]] = None, P: Optional[int] = None, device=None,
                 optimizer=None):
        if (params is None) == (optimizer is None):
            raise ValueError("ReferenceExchange: give either the optimizer (recommended) or a fixed params list")
        if params is not None and P is None:
            raise ValueError("ReferenceExchange: a fixed params list needs P")
        self.optimizer = optimizer
        self.fixed = None if params is None else list(params)
        self.fixed_sizes = None if params is None else [p.numel() for p in self.fixed]
        self.fixed_P = None if P is None else int(P)
        self.device = device
        self.flat = None
        self.params, self.sizes, self.n, self.P = [], [], -1, -1
        self.pending = False  # statistics deltas added since the last exchange
        if self.fixed is not None:
            self._bind(self.fixed_P)

    def _current(self) -> List[torch.Tensor]:
        if self.optimizer is not None:
            return [p for grp in self.optimizer.param_groups for p in grp["params"] if p.requires_grad]
        if any(p.numel() != n for p, n in zip(self.fixed, self.fixed_sizes)):
            raise RuntimeError("ReferenceExchange: a listed parameter changed size (densify_and_prune replaced "
                               "it): rebuild the exchange, or build it from the optimizer")
        return self.fixed

    def _bind(self, P: int) -> None:
        """(Re)lay out the bucket [gradients | one has-gradient flag per parameter | accum deltas |
        denom deltas] for the current parameters and P statistics rows."""
        if self.fixed_P is not None and P != self.fixed_P:
            raise RuntimeError(f"ReferenceExchange: the statistics hold {P} rows, the exchange was built for "
                               f"{self.fixed_P} (densify_and_prune resized them): rebuild it, or build it from the "
                               "optimizer")
        params = self._current()
        sizes = [p.numel() for p in params]
        n = sum(sizes) + len(params)
        if self.flat is None or n != self.n or P != self.P:
            if self.pending:
                raise RuntimeError("ReferenceExchange: the parameters or the statistics changed size between "
                                   "add_views and exchange")
            dev = self.device if self.device is not None else (params[0].device if params else "cpu")
            self.flat = torch.zeros(n + 2 * P, device=dev)
            self.acc = self.flat[n:n + P].view(P, 1)
            self.den = self.flat[n + P:].view(P, 1)
        self.params, self.sizes, self.n, self.P = params, sizes, n, P
        self.flags = self.flat[n - len(params):n]

    def add_views(self, mean2D_grads, radii, max_radii2D: torch.Tensor, stats_on: bool) -> None:
        """This rank's views' densification updates (train.py:130, 143-144)."""
        self._bind(int(max_radii2D.shape[0]))
        add_views(self.acc if stats_on else None, self.den if stats_on else None, max_radii2D, mean2D_grads, radii)
        self.pending = self.pending or stats_on

    def exchange(self, gaussians, stats_on: bool, world: int = 1, group=None, chunks: int = None,
                 min_chunk: int = None) -> int:
        """Sum the parameters' gradients (in place) and the statistics deltas over the ranks
        with one all-reduce; fold the deltas into gaussians.xyz_gradient_accum / denom.
        Returns the number of collectives issued."""
        P = int(gaussians.max_radii2D.shape[0])
        self._bind(P)
        if stats_on and (gaussians.xyz_gradient_accum.shape[0] != P or gaussians.denom.shape[0] != P):
            raise RuntimeError("ReferenceExchange: xyz_gradient_accum / denom do not hold max_radii2D's rows")
        o = 0
        for i, (p, n) in enumerate(zip(self.params, self.sizes)):
            if p.grad is not None:
                self.flat[o:o + n].copy_(p.grad.reshape(-1))
            else:  # no gradient on this rank (e.g. an embedding no local view used): adds zero
                self.flat[o:o + n].zero_()
            o += n
        self.flags.copy_(torch.tensor([0.0 if p.grad is None else 1.0 for p in self.params]))
        bucket = self.flat if stats_on else self.flat[:self.n]
        issued = 0
        if world > 1:
            ranges = exchange_chunks(bucket.numel(), EXCHANGE_CHUNKS if chunks is None else chunks,
                                     EXCHANGE_MIN_CHUNK if min_chunk is None else min_chunk)
            works = [dist.all_reduce(bucket[lo:hi], op=dist.ReduceOp.SUM, group=group, async_op=True)
                     for lo, hi in ranges]
            for w in works:
                w.wait()
            issued = len(ranges)
        o = 0
        anyg = self.flags.tolist() if world > 1 else None
        for i, (p, n) in enumerate(zip(self.params, self.sizes)):
            summed = self.flat[o:o + n].view_as(p)
            if p.grad is not None:
                p.grad.copy_(summed)
            elif anyg is not None and anyg[i] > 0:  # another rank's views reached it: every replica steps
                p.grad = summed.clone()
            o += n
        if stats_on:
            gaussians.xyz_gradient_accum.add_(self.acc)
            gaussians.denom.add_(self.den)
        self.acc.zero_()
        self.den.zero_()
        self.pending = False
        return issued


def shared_seed(group=None, device="cpu") -> int:
    """A fresh 63-bit seed drawn on rank 0 and broadcast to every rank."""
    seed = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64)
    if dist.is_available() and dist.is_initialized():
        t = seed.to(device)
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        seed = t.cpu()
    return int(seed.item())


def shared_generator(device, group=None) -> torch.Generator:
    """A generator on ``device`` seeded identically on every rank (the split's samples,
    gaussian_model.py:560)."""
    dev = torch.device(device)
    return torch.Generator(device=dev).manual_seed(shared_seed(group, dev if dev.type == "cuda" else "cpu"))


@contextlib.contextmanager
def consistent_rng(device, group=None):
    """Run the reference's own GaussianModel.densify_and_prune (which draws from the global
    RNG through torch.normal) with the global generators seeded identically on every rank,
    restoring them afterwards::

        with dp.consistent_rng("cuda", group):
            gaussians.densify_and_prune(...)
    """
    dev = torch.device(device)
    seed = shared_seed(group, dev if dev.type == "cuda" else "cpu")
    devices = [dev.index or 0] if dev.type == "cuda" else []
    with torch.random.fork_rng(devices=devices):
        torch.manual_seed(seed)
        yield seed


def replicas_identical(tensors: Sequence[torch.Tensor], group=None) -> List[bool]:
    """Whether every rank holds byte-identical ``tensors`` (a debug check after
    densification): each tensor's bytes are all-gathered (after its shape) and compared with
    rank 0's by ``torch.equal`` on the raw bytes, so NaN payloads, -0/+0 and any other bit
    difference count.  Returns one flag per tensor, the same on every rank."""
    if not (dist.is_available() and dist.is_initialized()):
        return [True for _ in tensors]
    world = dist.get_world_size(group)
    out = []
    for t in tensors:
        b = t.detach().contiguous().reshape(-1).view(torch.uint8)
        n = torch.tensor([b.numel()], dtype=torch.int64, device=b.device)
        ns = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(ns, n, group=group)
        if any(int(x) != int(n) for x in ns):
            out.append(False)
            continue
        bs = [torch.empty_like(b) for _ in range(world)]
        dist.all_gather(bs, b, group=group)
        out.append(all(torch.equal(bs[0], x) for x in bs[1:]))
    return out
