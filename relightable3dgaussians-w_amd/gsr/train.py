"""The data-parallel relightable training step (BASELINE cfg 4).

The reference trains on one view per iteration (train.py:56-194): environment SH from the
view's embedding, render(), the reconstruction / sky-BRDF / normal losses, backward,
densification statistics, one torch.optim.Adam step over nine param groups
(gaussian_model.py:259-274, relit3DGW_model.py:149).  The MI355X design:

  * every per-Gaussian attribute and the per-view lighting live in ONE flat fp32 buffer
    (FlatParams); each attribute is a leaf view of it, and each leaf's ``.grad`` is set to
    the matching view of ONE flat gradient buffer, so autograd accumulates in place and the
    gradient bucket needs no pack/unpack copies;
  * each rank renders its own views through the fused path (gsr.relit.render: relit
    features + one multi-channel composite + the image-space tail), ``views_per_rank`` of
    them per iteration, accumulating gradients;
  * one RCCL all-reduce (SUM) of the flat gradient buffer, one SUM/MAX of the
    densification statistics (gsr.dp) -- the path's only exchange steps;
  * one fused Adam launch over the flat buffer (gsr_adam_step): the per-group learning rates
    come from a segment table, and the all-reduced sum is turned into the mean over the
    step's views by the kernel's grad scale.

The iteration is the reference's (train.py:62-120): the view's embedding row through MLPNet
(scene/net_models.py:16-52, dropout in training mode) gives the environment SH (+ N(0, 0.025)
noise) and the sky SH; the losses are the reconstruction, sky-BRDF and normal terms plus the
envlight (envl_sh_loss), min-scale and sky-depth regularisers with the configured weights
(configs/optimizer/optimization_params.yaml).  The embedding table and the MLP weights are
segments of the same flat buffer, so their gradients cross the ranks in the same all-reduce.

Sky Gaussians are parametrised as the reference's: two angles (theta, phi) per sky Gaussian
on a shell of learnable radius around a fixed centre (gaussian_model.py:84-103,159-169,
227-251), so the gradient bucket carries xyz for the foreground and 2 floats per sky
Gaussian.  The loss terms switch on at the reference's iterations
(reg_normal_from_iter, reg_sky_gauss_depth_from_iter; train.py:89,113), and the envlight term
is added unweighted when lambda_envlight > 0 (train.py:99-102: the weight is only a switch).

Difference kept on purpose: the random draws (dropout masks, SH noise, envlight directions)
come from one device generator per scene instead of the global CPU/GPU RNG, so a step is
reproducible and synchronisation-free.
"""
from __future__ import annotations

import math
import types
from typing import Dict, List, Sequence, Tuple

import torch
import torch.nn.functional as F

from . import _lib

# (name, columns, lr) -- configs/optimizer/*.yaml defaults, in training_setup's group order
# (gaussian_model.py:259-274; xyz, scaling and sky_angles lrs carry the scene's spatial_lr_scale)
GAUSSIAN_GROUPS = (("xyz", 3, 0.00016), ("albedo", 3, 0.0025), ("opacity", 1, 0.05), ("scaling", 3, 0.001),
                   ("rotation", 4, 0.001), ("roughness", 1, 0.0002), ("metalness", 1, 0.0002),
                   ("sky_radius", 1, 0.0001), ("sky_angles", 2, 0.00016))
FG_ROW_GROUPS = ("xyz", "albedo", "roughness", "metalness")  # one row per foreground Gaussian
SKY_ROW_GROUPS = ("sky_angles",)                             # one row per sky Gaussian
SCENE_GROUPS = ("sky_radius",)                               # one value per scene
MLP_LR = 0.0002         # mlp_lr (configs/optimizer/optimization_params.yaml)
EMBEDDINGS_LR = 0.0002  # embeddings_lr
EMBEDDING_DIM = 32      # configs/relightable3DG-W.yaml embeddings_dim
# MLPNet(sh_degree_envl=4, sh_degree_sky=1, embedding_dim=32, dense_layer_size=256)
# (scene/net_models.py:16-40): (parameter name as in the reference's state_dict, out, in)
MLP_LAYERS = (("base.0", 256, 32), ("base.3", 256, 256), ("base.5", 128, 256), ("sh_sky_outlayer", 12, 128),
              ("sh_envl_layers.0", 128, 128), ("sh_envl_outlayer", 75, 128))
MLP_DROPOUT = 0.2
ENV_NOISE_STD = 0.025   # train.py:70
# loss weights (configs/optimizer/optimization_params.yaml)
LAMBDA_DSSIM, LAMBDA_SKY_BRDF, LAMBDA_NORMAL = 0.2, 0.5, 0.05
LAMBDA_ENVLIGHT, LAMBDA_SCALE, LAMBDA_SKY_GAUSS = 100.0, 100.0, 0.05
REG_NORMAL_FROM_ITER, REG_SKY_GAUSS_DEPTH_FROM_ITER = 15000, 0
# the position learning-rate schedule (configs/optimizer/optimization_params.yaml:4-7)
POSITION_LR_INIT, POSITION_LR_FINAL, POSITION_LR_DELAY_MULT, POSITION_LR_MAX_STEPS = 0.00016, 0.0000016, 0.01, 30000
MLP_LR_DROP_ITER, MLP_LR_AFTER_DROP = 20000, 0.0002  # relit3DGW_model.py:153-158


def expon_lr(step, lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000) -> float:
    """utils/general_utils.py:46-80 get_expon_lr_func's helper: log-linear from lr_init (step 0)
    to lr_final (max_steps), with the optional reverse-cosine delay, in double precision."""
    if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
        return 0.0
    if lr_delay_steps > 0:
        delay = lr_delay_mult + (1 - lr_delay_mult) * math.sin(0.5 * math.pi * min(max(step / lr_delay_steps, 0.0),
                                                                                   1.0))
    else:
        delay = 1.0
    t = min(max(step / max_steps, 0.0), 1.0)
    return delay * math.exp(math.log(lr_init) * (1 - t) + math.log(lr_final) * t)


def apply_lr_schedule(scene, iteration: int) -> None:
    """The learning rates the reference's Adam step of ``iteration`` uses (train.py:156-159 steps,
    then calls update_learning_rate(iteration) for the next one): xyz and sky_angles follow
    get_expon_lr_func at iteration - 1 (gaussian_model.py:277-293; its value at 0 is
    training_setup's initial rate), and the MLP / embedding groups are set to 0.0002 once
    iteration 20000 has stepped (relit3DGW_model.py:153-158).  Stateless: any iteration may be
    the first one run."""
    s = scene.spatial_lr_scale
    lr = expon_lr(iteration - 1, POSITION_LR_INIT * s, POSITION_LR_FINAL * s, lr_delay_mult=POSITION_LR_DELAY_MULT,
                  max_steps=POSITION_LR_MAX_STEPS)
    fp = scene.fp
    fp.set_lr("xyz", lr)
    fp.set_lr("sky_angles", lr)
    if iteration - 1 >= MLP_LR_DROP_ITER:
        for n in fp.names:
            if n == "embeddings" or n.startswith("mlp."):
                fp.set_lr(n, MLP_LR_AFTER_DROP)


class FlatParams:
    """Named fp32 parameters packed back to back (16-B aligned segments) in one buffer.

    ``params[name]`` is a leaf view of ``flat`` with ``.grad`` preset to the matching view
    of ``grad``; ``step()`` is one fused Adam launch (torch.optim.Adam semantics, eps as the
    reference's 1e-15).  ``tail`` extra floats follow ``grad`` in the same storage
    (``grad_tail``): the data-parallel step carries its densification sums there, so one
    all-reduce of ``bucket(True)`` moves both (gsr.dp.exchange)."""

    def __init__(self, spec: Sequence[Tuple[str, Tuple[int, ...], float]], device, betas=(0.9, 0.999), eps=1e-15,
                 tail: int = 0):
        self.names, self.shapes, self.lrs, self.offsets, ends = [], [], [], [], []
        o = 0
        for name, shape, lr in spec:
            n = int(math.prod(shape))
            self.names.append(name)
            self.shapes.append(tuple(shape))
            self.lrs.append(float(lr))
            self.offsets.append(o)
            o += (n + 3) // 4 * 4  # padding belongs to this segment (zero grads: no update)
            ends.append(o)
        self.n = o
        self.ends = ends
        self.device = torch.device(device)
        self.flat = torch.zeros(self.n, device=self.device)
        self.tail = int(tail)
        self._gstore = torch.zeros(self.n + self.tail, device=self.device)
        self.grad = self._gstore[:self.n]
        self.grad_tail = self._gstore[self.n:]
        self.exp_avg = torch.zeros(self.n, device=self.device)
        self.exp_avg_sq = torch.zeros(self.n, device=self.device)
        self.betas, self.eps, self.t = betas, eps, 0
        self.params: Dict[str, torch.Tensor] = {}
        for name, shape, off in zip(self.names, self.shapes, self.offsets):
            n = int(math.prod(shape))
            p = self.flat[off:off + n].view(shape)
            p.requires_grad_(True)
            p.grad = self.grad[off:off + n].view(shape)
            self.params[name] = p

    def load(self, name: str, value: torch.Tensor) -> None:
        with torch.no_grad():
            self.params[name].copy_(value.reshape(self.params[name].shape))

    def zero_grad(self, keep: Sequence[str] = ()) -> None:
        """Zero the gradient.  keep: segments this step's producers overwrite whole (the fused
        activations' backward): the zeroing starts at the first segment not kept (one fill of
        the buffer's tail instead of all of it; kept segments past that point are zeroed too,
        harmlessly)."""
        lo = min((o for n, o in zip(self.names, self.offsets) if n not in keep), default=self.n)
        # the kept segments must be a prefix (GAUSSIAN_GROUPS' order): one behind a zeroed
        # segment would be zeroed too, and a reordering would silently change what is kept
        assert all(o < lo for n, o in zip(self.names, self.offsets) if n in keep), \
            "zero_grad: a kept segment lies behind the first zeroed one"
        self._gstore[lo:].zero_()  # the tail too: this step's densification sums start at 0

    def bucket(self, with_tail: bool = False) -> torch.Tensor:
        """The flat gradient as one contiguous tensor, with the tail (``with_tail``) or not."""
        return self._gstore if with_tail else self.grad

    def check_grads_in_place(self) -> None:
        """Autograd accumulated into the preset views (not into fresh tensors)."""
        for name, off in zip(self.names, self.offsets):
            g = self.params[name].grad
            if self.params[name].numel() == 0:  # an empty group (no sky): nothing to accumulate
                continue
            if g is None or g.data_ptr() != self.grad.data_ptr() + 4 * off:
                raise RuntimeError(f"gradient of {name} left the flat buffer")

    def set_lr(self, name: str, lr: float) -> None:
        self.lrs[self.names.index(name)] = float(lr)

    def step(self, grad_scale: float = 1.0) -> None:
        self.begin_step(grad_scale)
        self.step_range(0, self.n)

    def begin_step(self, grad_scale: float = 1.0) -> None:
        """Start one Adam step (the step count, the groups' learning rates as they are now);
        step_range then applies it to element ranges, in any order, each exactly once."""
        import ctypes as C
        if self.device.type != "cuda":
            raise RuntimeError("FlatParams.step runs the HIP Adam kernel; parameters must be on the GPU")
        self.t += 1
        nseg = len(self.names)
        self._pending = ((C.c_longlong * nseg)(*self.ends), (C.c_double * nseg)(*self.lrs), nseg, float(grad_scale))

    def step_range(self, lo: int, hi: int) -> None:
        """The current step's update over elements [lo, hi) (lo a multiple of 4)."""
        ends, lrs, nseg, gs = self._pending
        hi = min(int(hi), self.n)
        if hi <= lo:
            return
        _lib.check(_lib.lib().gsr_adam_step_range(self.n, int(lo), hi, nseg, ends, lrs, self.betas[0], self.betas[1],
                                                  self.eps, self.t, gs, self.flat.data_ptr(), self.grad.data_ptr(),
                                                  self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
                                                  _lib.stream_of(self.device)), "gsr_adam_step_range")
        # the kernel wrote through a raw pointer: advance the version counter (shared by every
        # view of the flat buffer) so saved-tensor checks and version-keyed caches see it
        torch.autograd.graph.increment_version(self.flat)


# ---- losses (utils/loss_utils.py; the caller's code, restated for the step) ---------------

def l1_loss(out, gt, mask=None):
    """utils/loss_utils.py:27-35 (masked: sum |out*m - gt*m| / #(m == 1); 0 for an empty mask,
    as the reference's early return, without its host synchronisation)."""
    if mask is None:
        return (out - gt).abs().mean()
    n = (mask == 1).sum()
    s = (out * mask - gt * mask).abs().sum()
    return torch.where(n > 0, s / n.clamp(min=1), torch.zeros_like(s))


_WINDOWS: Dict[Tuple, torch.Tensor] = {}


def gaussian_1d(size=11, sigma=1.5):
    """utils/loss_utils.py:45-47: the fp32 window weights exp(-(x - 5)^2 / 4.5), normalised in fp32."""
    g = torch.tensor([math.exp(-(x - size // 2) ** 2 / float(2 * sigma ** 2)) for x in range(size)],
                     dtype=torch.float32)
    return g / g.sum()


def _window(size, channel, device):
    """utils/loss_utils.py:50-54: the 2-D depthwise window (outer product of gaussian_1d)."""
    key = (size, channel, str(device))
    if key not in _WINDOWS:
        g = gaussian_1d(size).unsqueeze(1)
        _WINDOWS[key] = (g @ g.t()).float().expand(channel, 1, size, size).contiguous().to(device)
    return _WINDOWS[key]


_WIN11 = None


class _FusedSSIM(torch.autograd.Function):
    """sum(ssim_map * mask) over the image (gsr_ssim_forward / gsr_ssim_backward); the
    gradient goes to img1 only (img2 is the ground truth)."""

    @staticmethod
    def forward(ctx, img1, img2, mask):
        import ctypes as C
        global _WIN11
        if _WIN11 is None:
            _WIN11 = (C.c_float * 11)(*gaussian_1d(11).tolist())
        Cn, H, W = img1.shape
        img1, img2 = img1.contiguous(), img2.contiguous()
        cstride = 0
        if mask is not None:
            mask = mask.float().contiguous()
            if mask.shape[0] == Cn and Cn > 1:
                cstride = H * W
        L = _lib.lib()
        parts = torch.empty((L.gsr_ssim_partials(Cn, H, W), 2), device=img1.device)
        dmaps = torch.empty((3, Cn, H, W), device=img1.device) if ctx.needs_input_grad[0] else None
        _lib.check(L.gsr_ssim_forward(Cn, H, W, img1.data_ptr(), img2.data_ptr(),
                                      None if mask is None else mask.data_ptr(), cstride, _WIN11, parts.data_ptr(),
                                      None if dmaps is None else dmaps.data_ptr(), _lib.stream_of(img1.device)),
                   "gsr_ssim_forward")
        ctx.save_for_backward(img1, img2, dmaps)
        # sum(map * mask) and #(mask == 1) over the C planes the kernel read; double keeps the
        # count exact past 2^24 elements (4K frames)
        sums = parts.double().sum(0)
        value, count = sums[0].float(), sums[1].clone()
        ctx.mark_non_differentiable(count)
        return value, count

    @staticmethod
    def backward(ctx, g, _g_count):
        img1, img2, dmaps = ctx.saved_tensors
        Cn, H, W = img1.shape
        gs = g.reshape(1).float().contiguous()
        d = torch.empty_like(img1)
        _lib.check(_lib.lib().gsr_ssim_backward(Cn, H, W, img1.data_ptr(), img2.data_ptr(), dmaps.data_ptr(),
                                                gs.data_ptr(), _WIN11, d.data_ptr(), 0, _lib.stream_of(img1.device)),
                   "gsr_ssim_backward")
        return d, None, None


def ssim(img1, img2, mask=None, window_size=11):
    """utils/loss_utils.py:53-96 (window 11, size_average): the masked mean of the SSIM map,
    on the fused HIP kernels.  Shapes [C,H,W] (a leading batch of 1 is squeezed, as the
    reference does); mask [C,H,W] or [1,H,W].  No host synchronisation: an empty mask gives
    1, as the reference's early return."""
    if window_size != 11:
        raise NotImplementedError("the fused SSIM implements the reference's 11x11 window")
    img1, img2 = img1.squeeze(0) if img1.dim() == 4 else img1, img2.squeeze(0) if img2.dim() == 4 else img2
    _lib.require_gpu_tensor(img1, "img1")
    _lib.require_gpu_tensor(img2, "img2")
    if img1.dim() != 3 or img1.shape != img2.shape:
        raise ValueError(f"ssim: images must both be [C,H,W], got {tuple(img1.shape)} and {tuple(img2.shape)}")
    if mask is not None:
        mask = mask.squeeze(0) if mask.dim() == 4 else mask
        C, H, W = img1.shape
        if mask.dim() != 3 or tuple(mask.shape[1:]) != (H, W) or mask.shape[0] not in (1, C):
            raise ValueError(f"ssim: mask must be [C,H,W] or [1,H,W], got {tuple(mask.shape)}")
        _lib.require_gpu_tensor(mask, "mask")
    # the kernel also counts #(mask == 1) over every plane it reads (a [1,H,W] mask stands
    # for its expansion over C, as the reference expands it)
    s, count = _FusedSSIM.apply(img1.float(), img2.float().detach(), None if mask is None else mask.detach())
    if mask is None:
        return s / img1.numel()
    return torch.where(count > 0, s / count.clamp(min=1), torch.ones_like(s)).to(s.dtype)


class _FusedViewLoss(torch.autograd.Function):
    """(1 - l_dssim) L1(img, gt; occ) + l_sky (L1(diff, 0; 1 - sky) + L1(spec, 0; 1 - sky))
    + l_normal mean(1 - sum_c (n o s)(nr o s)) on gsr_view_loss_forward/backward; masks [H,W]."""

    @staticmethod
    def forward(ctx, img, diff, spec, nrm, nref, gt, sky, occ, lam):
        H, W = sky.shape
        npix = H * W
        ts = [t.float().contiguous() for t in (img, gt, diff, spec, nrm, nref, sky, occ)]
        L = _lib.lib()
        parts = torch.empty((L.gsr_view_loss_partials(npix), 5), device=img.device)
        _lib.check(L.gsr_view_loss_forward(npix, *[t.data_ptr() for t in ts], parts.data_ptr(),
                                           _lib.stream_of(img.device)), "gsr_view_loss_forward")
        S = parts.double().sum(0)  # counts stay exact in double
        l_dssim, l_sky, l_normal = lam
        zero = torch.zeros((), dtype=torch.float64, device=img.device)
        k0 = torch.where(S[1] > 0, (1.0 - l_dssim) / S[1].clamp(min=1), zero)
        k2 = torch.where(S[3] > 0, l_sky / S[3].clamp(min=1), zero)
        loss = k0 * S[0] + k2 * S[2] + l_normal * (1.0 - S[4] / npix)
        ctx.coef = torch.stack([k0, k2, zero - l_normal / npix]).float()
        ctx.save_for_backward(*ts)
        return loss.float()

    @staticmethod
    def backward(ctx, g):
        ts = ctx.saved_tensors
        H, W = ts[6].shape
        coef = (ctx.coef * g.float()).contiguous()
        need = ctx.needs_input_grad
        outs = [torch.empty_like(ts[0]) if need[k] else None for k in range(5)]
        ptr = lambda t: None if t is None else t.data_ptr()
        _lib.check(_lib.lib().gsr_view_loss_backward(H * W, *[t.data_ptr() for t in ts], coef.data_ptr(),
                                                     *[ptr(t) for t in outs], _lib.stream_of(ts[0].device)),
                   "gsr_view_loss_backward")
        return (*outs, None, None, None, None)


def _plane(mask, H, W):
    """A [H,W] plane of a [H,W], [1,H,W] or channel-expanded [C,H,W] mask (channels equal)."""
    m = mask.detach()
    while m.dim() > 2:
        m = m[0]
    if tuple(m.shape) != (H, W):
        raise ValueError(f"mask shape {tuple(mask.shape)} does not match the image {H}x{W}")
    return m


class _FusedViewObjective(torch.autograd.Function):
    """The whole per-view objective of train.py:77-99 (pointwise terms + lambda_dssim
    (1 - SSIM(img, gt; occ))) in four launches forward (pointwise partials, SSIM partials
    and maps, gsr_view_objective for the scalar tail) and three backward (the coefficients
    times the upstream gradient, the pointwise gradients, the SSIM gradient added onto the
    image's), with no PyTorch scalar ops in between; equal to _FusedViewLoss + ssim()."""

    @staticmethod
    def forward(ctx, img, diff, spec, nrm, nref, gt, sky, occ, lam):
        import ctypes as C
        global _WIN11
        if _WIN11 is None:
            _WIN11 = (C.c_float * 11)(*gaussian_1d(11).tolist())
        H, W = sky.shape
        npix = H * W
        ts = [t.float().contiguous() for t in (img, gt, diff, spec, nrm, nref, sky, occ)]
        L = _lib.lib()
        dev = img.device
        st = _lib.stream_of(dev)
        nvl = L.gsr_view_loss_partials(npix)
        nss = L.gsr_ssim_partials(3, H, W)
        parts = torch.empty(5 * nvl + 2 * nss + 5, device=dev)
        vl, ss, loss, coef = parts[:5 * nvl], parts[5 * nvl:5 * nvl + 2 * nss], parts[-5:-4], parts[-4:]
        _lib.check(L.gsr_view_loss_forward(npix, *[t.data_ptr() for t in ts], vl.data_ptr(), st),
                   "gsr_view_loss_forward")
        dmaps = torch.empty((3, 3, H, W), device=dev) if ctx.needs_input_grad[0] else None
        _lib.check(L.gsr_ssim_forward(3, H, W, ts[0].data_ptr(), ts[1].data_ptr(), ts[7].data_ptr(), 0, _WIN11,
                                      ss.data_ptr(), None if dmaps is None else dmaps.data_ptr(), st),
                   "gsr_ssim_forward")
        _lib.check(L.gsr_view_objective(nvl, vl.data_ptr(), nss, ss.data_ptr(), npix, *[float(x) for x in lam],
                                        loss.data_ptr(), coef.data_ptr(), st), "gsr_view_objective")
        ctx.coef = coef
        ctx.dmaps = dmaps
        ctx.dest = (img, diff, spec)  # render()'s composite groups write into its GradSlab
        ctx.save_for_backward(*ts)
        return loss.view(())

    @staticmethod
    def backward(ctx, g):
        ts = ctx.saved_tensors
        H, W = ts[6].shape
        cg = (ctx.coef * g.float()).contiguous()  # (k_img, k_brdf, k_normal, k_ssim) x dL/dloss
        from .relit import slab_take
        need = ctx.needs_input_grad
        outs = []
        for k in range(5):
            d = None
            if need[k]:
                d = slab_take(ctx.dest[k]) if k < 3 else None
                if d is None or d.shape != ts[0].shape:
                    d = torch.empty_like(ts[0])
            outs.append(d)
        ptr = lambda t: None if t is None else t.data_ptr()
        st = _lib.stream_of(ts[0].device)
        # the image gradient (L1 + SSIM terms) in the SSIM backward's one pass; the other four here
        _lib.check(_lib.lib().gsr_view_loss_backward(H * W, *[t.data_ptr() for t in ts], cg.data_ptr(), None,
                                                     *[ptr(t) for t in outs[1:]], st), "gsr_view_loss_backward")
        if outs[0] is not None:
            _lib.check(_lib.lib().gsr_ssim_l1_backward(3, H, W, ts[0].data_ptr(), ts[1].data_ptr(), ctx.dmaps.data_ptr(),
                                                       cg.data_ptr() + 12, _WIN11, ts[7].data_ptr(), cg.data_ptr(),
                                                       outs[0].data_ptr(), st), "gsr_ssim_l1_backward")
        return (*outs, None, None, None, None)


def view_loss(out, gt, sky_mask, occ_mask, lambda_dssim=0.2, lambda_sky_brdf=0.5, lambda_normal=0.05):
    """train.py:77-99: reconstruction (L1 + D-SSIM), sky-BRDF and normal-consistency terms,
    fused (_FusedViewObjective: gsr_view_loss_*, gsr_ssim_*, gsr_view_objective).  Masks:
    [H,W], [1,H,W] or their channel expansion."""
    img = out["render"]
    H, W = img.shape[-2:]
    sky, occ = _plane(sky_mask, H, W), _plane(occ_mask, H, W)
    _lib.require_gpu_tensor(img, "render")
    if img.dim() != 3 or img.shape[0] != 3 or gt.shape != img.shape:
        raise ValueError(f"view_loss: render and gt must both be [3,H,W], got {tuple(img.shape)}, {tuple(gt.shape)}")
    return _FusedViewObjective.apply(img, out["diffuse_color"], out["specular_color"], out["normal"],
                                     out["normal_ref"], gt.detach(), sky, occ,
                                     (float(lambda_dssim), float(lambda_sky_brdf), float(lambda_normal)))


def view_loss_unfused(out, gt, sky_mask, occ_mask, lambda_dssim=0.2, lambda_sky_brdf=0.5, lambda_normal=0.05):
    """view_loss with the scalar tail in PyTorch (_FusedViewLoss + ssim()): the fused
    objective's test reference."""
    img = out["render"]
    H, W = img.shape[-2:]
    sky, occ = _plane(sky_mask, H, W), _plane(occ_mask, H, W)
    _lib.require_gpu_tensor(img, "render")
    pw = _FusedViewLoss.apply(img, out["diffuse_color"], out["specular_color"], out["normal"], out["normal_ref"],
                              gt.detach(), sky, occ, (float(lambda_dssim), float(lambda_sky_brdf),
                                                      float(lambda_normal)))
    return pw + lambda_dssim * (1.0 - ssim(img, gt, occ[None]))


def view_loss_torch(out, gt, sky_mask, occ_mask, lambda_dssim=0.2, lambda_sky_brdf=0.5, lambda_normal=0.05):
    """The same loss composed from PyTorch ops as train.py writes it (test reference for the
    fused kernels; its SSIM is the fused one)."""
    img = out["render"]
    rec = l1_loss(img, gt, occ_mask) * (1 - lambda_dssim) + lambda_dssim * (1.0 - ssim(img, gt, occ_mask))
    nsky = 1 - sky_mask
    loss = rec + lambda_sky_brdf * (l1_loss(out["diffuse_color"], torch.zeros_like(img), nsky) +
                                    l1_loss(out["specular_color"], torch.zeros_like(img), nsky))
    n = out["normal"] * occ_mask * sky_mask
    nr = out["normal_ref"] * occ_mask * sky_mask
    return loss + lambda_normal * (1 - (n * nr).sum(dim=0))[None].mean()


# ---- the environment-light MLP and the regularisers (train.py:66-120) ---------------------

def mlp_forward(params: Dict[str, torch.Tensor], emb: torch.Tensor, drop_mask=None):
    """MLPNet.forward (scene/net_models.py:43-52) on the named weights ``mlp.<layer>.weight``
    / ``.bias`` of ``params``: Linear(32, 256) -> Dropout(0.2) -> ReLU -> Linear(256, 256) ->
    ReLU -> Linear(256, 128) -> ReLU, then the sky head Linear(128, 12) and the environment head
    Linear(128, 128) -> ReLU -> Linear(128, 75).  ``drop_mask`` [B, 256]: the training-mode
    dropout multiplier (0 or 1/(1-p)); None is eval mode.  Returns (env [B,25,3], sky [B,4,3])."""
    def lin(x, name):
        return F.linear(x, params[f"mlp.{name}.weight"], params[f"mlp.{name}.bias"])
    h = lin(emb, "base.0")
    if drop_mask is not None:
        h = h * drop_mask
    h = F.relu(h)
    h = F.relu(lin(h, "base.3"))
    h = F.relu(lin(h, "base.5"))
    sky = lin(h, "sh_sky_outlayer").view(-1, 4, 3)
    env = lin(F.relu(lin(h, "sh_envl_layers.0")), "sh_envl_outlayer").view(-1, 25, 3)
    return env, sky


def sh_basis(deg: int, d: torch.Tensor) -> torch.Tensor:
    """The real SH basis of utils/sh_utils.py:81-151 (constants :35-64) at unit directions
    d [N,3], degrees 0-4: [N, (deg+1)^2], so eval_sh(deg, sh, d) = basis @ sh per channel."""
    if not 0 <= deg <= 4:
        raise ValueError("sh_basis: degrees 0-4")
    x, y, z = d[:, 0], d[:, 1], d[:, 2]
    b = [torch.full_like(x, 0.28209479177387814)]
    if deg > 0:
        c1 = 0.4886025119029199
        b += [-c1 * y, c1 * z, -c1 * x]
    if deg > 1:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        b += [1.0925484305920792 * xy, -1.0925484305920792 * yz, 0.31539156525252005 * (2.0 * zz - xx - yy),
              -1.0925484305920792 * xz, 0.5462742152960396 * (xx - yy)]
    if deg > 2:
        b += [-0.5900435899266435 * y * (3 * xx - yy), 2.890611442640554 * xy * z,
              -0.4570457994644658 * y * (4 * zz - xx - yy), 0.3731763325901154 * z * (2 * zz - 3 * xx - 3 * yy),
              -0.4570457994644658 * x * (4 * zz - xx - yy), 1.445305721320277 * z * (xx - yy),
              -0.5900435899266435 * x * (xx - 3 * yy)]
    if deg > 3:
        b += [2.5033429417967046 * xy * (xx - yy), -1.7701307697799304 * yz * (3 * xx - yy),
              0.9461746957575601 * xy * (7 * zz - 1), -0.6690465435572892 * yz * (7 * zz - 3),
              0.10578554691520431 * (zz * (35 * zz - 30) + 3), -0.6690465435572892 * xz * (7 * zz - 3),
              0.47308734787878004 * (xx - yy) * (7 * zz - 1), -1.7701307697799304 * xz * (xx - 3 * yy),
              0.6258357354491761 * (xx * (xx - 3 * yy) - yy * (3 * xx - yy))]
    return torch.stack(b, dim=-1)


def envl_sh_loss(sh_env: torch.Tensor, sh_degree: int, N_samples: int = 10, dirs: torch.Tensor = None,
                 generator: torch.Generator = None) -> torch.Tensor:
    """utils/loss_utils.py:185-207: the environment SH [1,K,3] evaluated at N_samples random
    directions (U(-1,1)^3 normalised; ``dirs`` [N_samples,3] supplies the unnormalised draw),
    and the mean squared negative part of the 3 N_samples values (0 when none is negative).
    No host synchronisation: the reference's boolean selection becomes a masked sum / count."""
    if dirs is None:
        dirs = torch.empty(N_samples, 3, device=sh_env.device).uniform_(-1, 1, generator=generator)
    d = dirs / dirs.norm(dim=1, keepdim=True)
    vals = sh_basis(sh_degree, d) @ sh_env.reshape(-1, 3)[: (sh_degree + 1) ** 2]  # [N, 3]
    neg = (vals < 0).to(vals.dtype)
    n = neg.sum()
    return torch.where(n > 0, (vals * vals * neg).sum() / n.clamp(min=1), torch.zeros_like(n))


def min_scale_loss(radii: torch.Tensor, gaussians) -> torch.Tensor:
    """utils/loss_utils.py:210-220: the mean over visible foreground Gaussians of their
    smallest scale (get_scaling sorted along the last axis, column 0); masked sum / count."""
    vis = (radii > 0) & ~gaussians.get_is_sky.reshape(-1)
    smin = gaussians.get_scaling.min(dim=-1).values
    w = vis.to(smin.dtype)
    return (smin * w).sum() / w.sum()


def depth_loss_gaussians(gaussians, camera, visibility_filter: torch.Tensor, gamma: float = 0.02) -> torch.Tensor:
    """utils/loss_utils.py:140-148: exp(-gamma (mean sky depth - mean foreground depth)) over
    the visible Gaussians, the foreground mean detached.  The view-space depth is the third
    column of the row-vector world-to-view matrix (GaussianModel.get_depth, :125-130),
    evaluated elementwise: a batched [4,4] x [P,4,1] matmul, or a [P,3] x [3] gemv (rocBLAS
    gemvt: 1.1 ms at P = 1.5M), costs more than the whole render of the view."""
    wvt = camera.world_view_transform
    x = gaussians.get_xyz
    depth = x[:, 0] * wvt[0, 2] + x[:, 1] * wvt[1, 2] + x[:, 2] * wvt[2, 2] + wvt[3, 2]
    sky = gaussians.get_is_sky.reshape(-1)
    ws = (sky & visibility_filter).to(depth.dtype)
    wf = (~sky & visibility_filter).to(depth.dtype)
    avg_sky = (depth * ws).sum() / ws.sum()
    avg_fg = ((depth * wf).sum() / wf.sum()).detach()
    return torch.exp(-gamma * (avg_sky - avg_fg))


REG_MAXV = 8  # views per launch of the fused regulariser passes (gsr::REG_MAXV, csrc/gsr_trainaux.hip)


class _FusedViewRegs(torch.autograd.Function):
    """The per-Gaussian half of view_regularisers as one HIP pass each way
    (csrc/gsr_trainaux.hip): sums [V,5] per view = (#visible foreground, #visible sky,
    sum min-scale over visible foreground, sum depth over visible sky, sum depth over visible
    foreground), differentiable in xyz and scaling."""

    @staticmethod
    def forward(ctx, xyz, scaling, dcol, radii, is_sky, sink_in=None):
        P, V = xyz.shape[0], len(radii)
        L = _lib.lib()
        parts = torch.empty(L.gsr_view_regularisers_partials(P), 5 * V, device=xyz.device)
        rp = _lib.ptr_array(radii)
        _lib.check(L.gsr_view_regularisers_forward(P, V, xyz.data_ptr(), scaling.data_ptr(), rp, is_sky.data_ptr(),
                                                   dcol.data_ptr(), parts.data_ptr(), _lib.stream_of(xyz.device)),
                   "gsr_view_regularisers_forward")
        ctx.save_for_backward(scaling, dcol, is_sky, *radii)
        ctx.P, ctx.V = P, V
        ctx.sink_in = sink_in or (None, None)  # the model's xyz and scaling (gsr.sink)
        return parts.sum(0).view(V, 5)

    @staticmethod
    def backward(ctx, g):
        from . import sink as gsink
        scaling, dcol, is_sky, *radii = ctx.saved_tensors
        need = ctx.needs_input_grad
        if not (need[0] or need[1]):
            return None, None, None, None, None, None
        outs, ret, sk, claimed, acc = gsink.outputs(ctx.sink_in, (need[0], need[1]))
        dx = outs[0] if outs[0] is not None else (torch.empty(ctx.P, 3, device=scaling.device) if need[0] else None)
        ds = outs[1] if outs[1] is not None else (torch.empty_like(scaling) if need[1] else None)
        ptr = lambda t: None if t is None else t.data_ptr()
        _lib.check(_lib.lib().gsr_view_regularisers_backward(ctx.P, ctx.V, scaling.data_ptr(), _lib.ptr_array(radii),
                                                             is_sky.data_ptr(), dcol.data_ptr(),
                                                             g.contiguous().data_ptr(), ptr(dx), ptr(ds), acc,
                                                             _lib.stream_of(scaling.device)),
                   "gsr_view_regularisers_backward")
        if sk is not None:
            sk.done(claimed)
        return (dx if ret[0] else None), (ds if ret[1] else None), None, None, None, None


def sh_basis_fused(deg: int, dirs: torch.Tensor) -> torch.Tensor:
    """sh_basis(deg, dirs / |dirs|) as one HIP launch (gsr_sh_basis); no gradient (the
    directions are random draws)."""
    N = dirs.shape[0]
    d = dirs.detach().float().contiguous()
    out = torch.empty(N, (deg + 1) ** 2, device=dirs.device)
    _lib.check(_lib.lib().gsr_sh_basis(N, deg, d.data_ptr(), out.data_ptr(), _lib.stream_of(dirs.device)),
               "gsr_sh_basis")
    return out


class _RegsTail(torch.autograd.Function):
    """view_regularisers' per-view scalar tail (gsr_view_regularisers_tail_*): the sums
    [V,5] of _FusedViewRegs, the environment SH [V,25,3] and the basis at the envlight
    directions -> total [V], one workgroup each way (the ~40 [V]-sized PyTorch ops of the
    composition, on the iteration's critical path between the views and the backward)."""

    @staticmethod
    def forward(ctx, sums, env_sh, basis, depth_on, gamma):
        V = sums.shape[0]
        ns = basis.shape[0] // V
        s_, e_, b_ = sums.float().contiguous(), env_sh.reshape(V, 25, 3).float().contiguous(), basis.contiguous()
        total = torch.empty(V, dtype=torch.float32, device=sums.device)
        consts = (float(LAMBDA_ENVLIGHT), float(LAMBDA_SCALE), float(LAMBDA_SKY_GAUSS), float(gamma), int(depth_on))
        _lib.check(_lib.lib().gsr_view_regularisers_tail_forward(V, ns, s_.data_ptr(), b_.data_ptr(), e_.data_ptr(),
                                                                 *consts, total.data_ptr(),
                                                                 _lib.stream_of(sums.device)),
                   "gsr_view_regularisers_tail_forward")
        ctx.save_for_backward(s_, e_, b_)
        ctx.consts, ctx.ns, ctx.env_shape = consts, ns, env_sh.shape
        return total

    @staticmethod
    def backward(ctx, g):
        s_, e_, b_ = ctx.saved_tensors
        V = s_.shape[0]
        d_sums = torch.empty_like(s_)
        d_env = torch.empty_like(e_)
        _lib.check(_lib.lib().gsr_view_regularisers_tail_backward(
            V, ctx.ns, s_.data_ptr(), b_.data_ptr(), e_.data_ptr(), *ctx.consts, g.float().contiguous().data_ptr(),
            d_sums.data_ptr(), d_env.data_ptr(), _lib.stream_of(s_.device)), "gsr_view_regularisers_tail_backward")
        return d_sums, d_env.view(ctx.env_shape), None, None, None


def view_regularisers(pc, radii, viewmats: torch.Tensor, env_sh: torch.Tensor, dirs: torch.Tensor,
                      gamma: float = 0.02, depth_on: bool = True, fused: bool = None,
                      tail_fused: bool = True) -> torch.Tensor:
    """The three regularisers of train.py:99-118 for V views at once, as [V] losses:
    envl_sh_loss(env_sh[v]) (unweighted: lambda_envlight only switches it on, :99-102)
    + LAMBDA_SCALE min_scale_loss(radii[v]) + LAMBDA_SKY_GAUSS depth_loss_gaussians(view v)
    (when ``depth_on``: iteration > reg_sky_gauss_depth_from_iter, :113), each equal to the
    single-view function above.  radii [V,P] or a list of V [P] tensors, viewmats [V,4,4]
    (row-vector world-to-view), env_sh [V,25,3], dirs [V,10,3].

    ``fused`` (default: on GPU tensors): the per-Gaussian sums of all V views in one HIP pass
    each way, the SH basis in one launch and (``tail_fused``) the scalar tail in one
    workgroup each way (csrc/gsr_trainaux.hip); otherwise the PyTorch composition below (~15
    [V,P] kernels each way plus V x 5 reductions), which is also the fused path's test
    reference."""
    V = len(radii)
    x = pc.get_xyz
    if fused is None:
        fused = x.is_cuda
    if fused and V > REG_MAXV:
        # the HIP passes take up to REG_MAXV views per launch; each view's terms are independent
        return torch.cat([view_regularisers(pc, radii[i:i + REG_MAXV], viewmats[i:i + REG_MAXV],
                                            env_sh[i:i + REG_MAXV], dirs[i:i + REG_MAXV], gamma, depth_on, fused,
                                            tail_fused) for i in range(0, V, REG_MAXV)])
    c = viewmats[:, :, 2]                                      # [V,4]: the depth column
    if fused:
        rl = [r.contiguous() for r in radii] if isinstance(radii, (list, tuple)) else list(radii.contiguous())
        sky_u8 = pc.get_is_sky.reshape(-1).contiguous()
        sums = _FusedViewRegs.apply((x if depth_on else x.detach()).contiguous(), pc.get_scaling.contiguous(),
                                    c.float().contiguous(), rl, sky_u8, (x if depth_on else None, pc.get_scaling))
        if tail_fused:  # the scalar tail and the envlight term in one launch each way
            basis = sh_basis_fused(4, dirs.reshape(-1, 3))
            return _RegsTail.apply(sums, env_sh, basis, bool(depth_on), float(gamma))
        nf, ns = sums[:, 0], sums[:, 1]
        ms = sums[:, 2] / nf
        avg_sky = sums[:, 3] / ns
        avg_fg = (sums[:, 4] / nf).detach()
    else:
        radii = torch.stack(list(radii)) if isinstance(radii, (list, tuple)) else radii

        def rows(t):  # per-view sums of a [V,P] tensor
            return torch.stack([t[v].sum() for v in range(V)])
        sky = pc.get_is_sky.reshape(-1)
        vis = radii > 0
        wf = (vis & ~sky).to(torch.float32)                        # visible foreground
        ws = (vis & sky).to(torch.float32)                         # visible sky
        nf, ns = rows(wf), rows(ws)
        smin = pc.get_scaling.min(dim=-1).values                   # [P]
        ms = rows(wf * smin) / nf
        depth = x[:, 0] * c[:, 0:1] + x[:, 1] * c[:, 1:2] + x[:, 2] * c[:, 2:3] + c[:, 3:4]   # [V,P]
        avg_sky = rows(depth * ws) / ns
        avg_fg = (rows(depth * wf) / nf).detach()
    dl = torch.exp(-gamma * (avg_sky - avg_fg))
    if fused:
        basis = sh_basis_fused(4, dirs.reshape(-1, 3))
    else:
        d = dirs / dirs.norm(dim=-1, keepdim=True)
        basis = sh_basis(4, d.reshape(-1, 3))
    vals = torch.bmm(basis.reshape(V, -1, 25), env_sh.reshape(V, 25, 3))  # [V,10,3]
    neg = (vals < 0).to(vals.dtype)
    n = neg.sum(dim=(1, 2))
    el = torch.where(n > 0, (vals * vals * neg).sum(dim=(1, 2)) / n.clamp(min=1), torch.zeros_like(n))
    total = torch.zeros_like(ms)
    if LAMBDA_ENVLIGHT > 0:
        total = total + el
    if LAMBDA_SCALE > 0:
        total = total + LAMBDA_SCALE * ms
    if depth_on and LAMBDA_SKY_GAUSS > 0:
        total = total + LAMBDA_SKY_GAUSS * dl
    return total


# ---- the sky Gaussians' parametrisation (gaussian_model.py:84-103,159-169) -----------------

def cartesian_to_polar_coord(xyz: torch.Tensor, center: torch.Tensor = None, radius=1.0) -> torch.Tensor:
    """utils/general_utils.py:295-299: theta = acos(clamp((c_y - y) / radius, -1, 1)),
    phi = atan2(x - c_x, z - c_z), as [N,2].  ``radius`` defaults to 1.0 as in the reference
    (densify_and_split calls it without a radius, gaussian_model.py:573)."""
    if center is None:
        center = torch.zeros(3, dtype=xyz.dtype, device=xyz.device)
    theta = torch.acos(torch.clamp((-xyz[..., 1] + center[1]) / radius, -1, 1)).unsqueeze(1)
    phi = torch.atan2(xyz[..., 0] - center[0], xyz[..., 2] - center[2]).unsqueeze(1)
    return torch.cat((theta, phi), dim=1)


def sky_angles_clamped(a: torch.Tensor) -> torch.Tensor:
    """get_sky_angles (gaussian_model.py:159-169): theta clamped to [0, pi/2], phi to
    [-pi/2, pi/2] (zero gradient outside the range)."""
    tm = (a[..., 0] < 0) | (a[..., 0] > torch.pi / 2)
    pm = (a[..., 1] < -torch.pi / 2) | (a[..., 1] > torch.pi / 2)
    th = torch.where(tm, torch.clamp(a[..., 0], 0, torch.pi / 2), a[..., 0])
    ph = torch.where(pm, torch.clamp(a[..., 1], -torch.pi / 2, torch.pi / 2), a[..., 1])
    return torch.cat((th.unsqueeze(1), ph.unsqueeze(1)), dim=1)


# the leading segments of GAUSSIAN_GROUPS that _Activations.backward overwrites whole every step
# (sky_angles is overwritten too but sits behind sky_radius, so zero_grad zeroes it)
_ACT_OVERWRITES = ("xyz", "albedo", "opacity", "scaling", "rotation", "roughness", "metalness")


class _Activations(torch.autograd.Function):
    """RelitScene's activations (gaussian_model.py:69-103) in one HIP pass each way
    (gsr_activations_forward / _backward).  The backward writes the raw parameters' gradients
    into the scene's flat gradient (their preset .grad views) and returns none to autograd,
    so no AccumulateGrad kernel runs for them; the parameters receive gradients from these
    activations only."""

    KEYS = ("xyz", "scaling", "rotation", "opacity", "albedo", "roughness", "metalness")

    @staticmethod
    def forward(ctx, scene, box, xyz_fg, angles, radius, scale_raw, rot_raw, op_raw, alb_raw, rough_raw, metal_raw):
        lay = scene.layout
        P, Nfg, Nsky = lay.P, lay.n_fg, lay.n_sky
        dev = xyz_fg.device
        f = dict(dtype=torch.float32, device=dev)
        xyz, scale, rot = torch.empty(P, 3, **f), torch.empty(P, 3, **f), torch.empty(P, 4, **f)
        op = torch.empty(P, 1, **f)
        alb, rough, metal = torch.empty(Nfg, 3, **f), torch.empty(Nfg, 1, **f), torch.empty(Nfg, 1, **f)
        center = scene.sky_center.float().contiguous()
        ins = [xyz_fg, angles, radius, center, scale_raw, rot_raw, op_raw, alb_raw, rough_raw, metal_raw]
        ptr = lambda t: None if t is None or t.numel() == 0 else t.data_ptr()
        src = None if lay.src is None else lay.src.data_ptr()
        _lib.check(_lib.lib().gsr_activations_forward(P, Nfg, Nsky, src, *[ptr(t) for t in ins],
                                                      *[ptr(t) for t in (xyz, scale, rot, op, alb, rough, metal)],
                                                      _lib.stream_of(dev)), "gsr_activations_forward")
        ctx.scene = scene
        ctx.box = box  # [GradSink]: set by model_fused once the outputs exist
        ctx.ins = ins
        ctx.outs = (scale, rot, op, alb, rough, metal)
        ctx.set_materialize_grads(False)
        return xyz, scale, rot, op, alb, rough, metal

    @staticmethod
    def backward(ctx, *g):
        scene = ctx.scene
        lay, fp = scene.layout, scene.fp
        P, Nfg, Nsky = lay.P, lay.n_fg, lay.n_sky
        dev = ctx.ins[0].device
        ptr = lambda t: None if t is None or t.numel() == 0 else t.data_ptr()
        gs = [None if t is None else t.float().contiguous() for t in g]
        sk = ctx.box[0]
        if sk is not None:  # the views' summed gradients (plus any autograd brought)
            for i, k in enumerate(_Activations.KEYS):
                b = sk.take(k)
                if b is not None:
                    gs[i] = b if gs[i] is None else gs[i] + b
        d = {n: fp.params[n].grad for n in ("xyz", "sky_angles", "sky_radius", "scaling", "rotation", "opacity",
                                             "albedo", "roughness", "metalness")}
        part = torch.empty(max(1, _lib.lib().gsr_activations_partials(P, Nfg)), dtype=torch.float32, device=dev)
        src = None if lay.src is None else lay.src.data_ptr()
        _lib.check(_lib.lib().gsr_activations_backward(
            P, Nfg, Nsky, src, *[ptr(t) for t in ctx.ins], *[ptr(t) for t in ctx.outs], *[ptr(t) for t in gs],
            ptr(d["xyz"]), ptr(d["sky_angles"]), ptr(d["sky_radius"]), part.data_ptr(), ptr(d["scaling"]),
            ptr(d["rotation"]), ptr(d["opacity"]), ptr(d["albedo"]), ptr(d["roughness"]), ptr(d["metalness"]),
            _lib.stream_of(dev)), "gsr_activations_backward")
        scene.act_grads_written = True  # train_step: the kept (unzeroed) segments hold this step's values
        return (None,) * 11


class _FusedSkyXYZ(torch.autograd.Function):
    """sky_xyz as one HIP pass each way (gsr_sky_xyz_forward/backward); differentiable in
    the angles and the radius (the centre is a constant of the scene)."""

    @staticmethod
    def forward(ctx, angles, radius, center):
        N = angles.shape[0]
        out = torch.empty(N, 3, device=angles.device)
        _lib.check(_lib.lib().gsr_sky_xyz_forward(N, angles.data_ptr(), radius.data_ptr(), center.data_ptr(),
                                                  out.data_ptr(), _lib.stream_of(angles.device)), "gsr_sky_xyz_forward")
        ctx.save_for_backward(angles, radius)
        return out

    @staticmethod
    def backward(ctx, g):
        angles, radius = ctx.saved_tensors
        N = angles.shape[0]
        L = _lib.lib()
        da = torch.empty_like(angles)
        dr = torch.empty(L.gsr_sky_xyz_partials(N), device=angles.device)
        _lib.check(L.gsr_sky_xyz_backward(N, angles.data_ptr(), radius.data_ptr(), g.contiguous().data_ptr(),
                                          da.data_ptr(), dr.data_ptr(), _lib.stream_of(angles.device)),
                   "gsr_sky_xyz_backward")
        return da, dr.sum().reshape(radius.shape), None


def sky_xyz(angles: torch.Tensor, radius: torch.Tensor, center: torch.Tensor, fused: bool = None) -> torch.Tensor:
    """get_sky_xyz (gaussian_model.py:95-103), COLMAP axes: radius (sin t sin p, -cos t,
    sin t cos p) + center, from the clamped angles.  ``fused`` (default: on GPU tensors):
    one HIP pass each way instead of ~20 elementwise kernels."""
    if fused is None:
        fused = angles.is_cuda
    if fused and angles.shape[0]:
        return _FusedSkyXYZ.apply(angles.contiguous(), radius.contiguous(), center.float().contiguous())
    a = sky_angles_clamped(angles)
    x = torch.sin(a[..., 0]) * torch.sin(a[..., 1])
    y = -torch.cos(a[..., 0])
    z = torch.sin(a[..., 0]) * torch.cos(a[..., 1])
    return radius * torch.stack([x, y, z], dim=-1) + center.reshape(-1)


class SkyLayout:
    """Where the foreground and sky rows sit among all P Gaussians (get_xyz's scatter by the
    sky flags, gaussian_model.py:84-93), as index tensors made once per scene layout (boolean
    indexing would synchronise with the host every iteration).  ``tail``: the sky Gaussians
    are the last rows, so the scatter is one concatenation."""

    def __init__(self, is_sky: torch.Tensor):
        m = is_sky.reshape(-1).bool()
        self.P = int(m.numel())
        self.n_sky = int(m.sum())
        self.n_fg = self.P - self.n_sky
        self.tail = bool(m[self.n_fg:].all()) and not bool(m[:self.n_fg].any())
        self.fg_idx = torch.nonzero(~m).reshape(-1)
        self.sky_idx = torch.nonzero(m).reshape(-1)
        # the fused activations' row map (gsr_activations_*): the foreground row, or -1 - the
        # sky row, per Gaussian; None for the tail layout
        self.src = None
        if self.n_sky and not self.tail:
            src = torch.empty(self.P, dtype=torch.int32, device=m.device)
            src[self.fg_idx] = torch.arange(self.n_fg, dtype=torch.int32, device=m.device)
            src[self.sky_idx] = -1 - torch.arange(self.n_sky, dtype=torch.int32, device=m.device)
            self.src = src

    def xyz(self, xyz_fg: torch.Tensor, xyz_sky: torch.Tensor) -> torch.Tensor:
        if self.n_sky == 0:
            return xyz_fg.view(xyz_fg.shape)
        if self.tail:
            return torch.cat([xyz_fg, xyz_sky], dim=0)
        out = torch.zeros(self.P, 3, dtype=xyz_fg.dtype, device=xyz_fg.device)
        return out.index_put((self.fg_idx,), xyz_fg).index_put((self.sky_idx,), xyz_sky)


def draw_step_randomness(n_views: int, device, generator: torch.Generator = None) -> Dict[str, torch.Tensor]:
    """The iteration's random draws for ``n_views`` views: MLPNet's dropout multipliers
    [V,256] (0 or 1/(1-p)), the environment SH noise [V,25,3] ~ N(0, 0.025) (train.py:70) and
    the envlight regulariser's unnormalised directions [V,10,3] ~ U(-1,1)."""
    keep = torch.rand(n_views, MLP_LAYERS[0][1], device=device, generator=generator) >= MLP_DROPOUT
    return {"dropout": keep.float() / (1.0 - MLP_DROPOUT),
            "noise": torch.randn(n_views, 25, 3, device=device, generator=generator) * ENV_NOISE_STD,
            "dirs": torch.rand(n_views, 10, 3, device=device, generator=generator) * 2.0 - 1.0}


# ---- the model view render() reads and the step ------------------------------------------

class RelitScene:
    """A relightable scene on one rank: FlatParams with the Gaussian groups (foreground xyz,
    sky (theta, phi) angles and the sky shell radius as the reference stores them), the
    per-view embedding table [n_views, 32] (relit3DGW_model.py:66-67) and MLPNet's weights
    (the ``mlp.*`` groups, PyTorch's default Linear initialisation), and the constant sky
    flags.  ``model()`` gives the activated attributes as render() reads them
    (gaussian_model.py:74-180: get_xyz scattered from the foreground rows and the shell, exp
    scaling, normalised rotation, sigmoid opacity and materials).

    ``xyz`` [P,3] are all positions; the sky rows become angles on a shell around
    ``sky_center`` (default: the origin) of radius ``sky_radius`` (default: the sky rows'
    median distance from the centre), as augment_with_sky_gaussians does (:227-251)."""

    def __init__(self, xyz, scaling_raw, rotation_raw, opacity_raw, albedo_raw, rough_raw, metal_raw, is_sky,
                 n_views, device, spatial_lr_scale=1.0, seed=0, sky_center=None, sky_radius=None):
        P, N_fg = xyz.shape[0], albedo_raw.shape[0]
        m = is_sky.reshape(-1).bool().cpu()
        if int((~m).sum()) != N_fg:
            raise ValueError(f"RelitScene: {int((~m).sum())} foreground Gaussians but {N_fg} material rows")
        self.sky_center = (torch.zeros(3) if sky_center is None else torch.as_tensor(sky_center).float().reshape(3))
        xyz = xyz.float().cpu()
        sky_pts = xyz[m]
        if sky_radius is None:
            sky_radius = float((sky_pts - self.sky_center).norm(dim=1).median()) if sky_pts.shape[0] else 1.0
        spec = []
        for name, cols, lr in GAUSSIAN_GROUPS:
            if name in ("xyz", "scaling", "sky_angles"):
                lr *= spatial_lr_scale
            rows = N_fg if name in FG_ROW_GROUPS else (P - N_fg) if name in SKY_ROW_GROUPS else P
            spec.append((name, (1,) if name in SCENE_GROUPS else (rows, cols), lr))
        spec.append(("embeddings", (n_views, EMBEDDING_DIM), EMBEDDINGS_LR))
        for name, fout, fin in MLP_LAYERS:
            spec += [(f"mlp.{name}.weight", (fout, fin), MLP_LR), (f"mlp.{name}.bias", (fout,), MLP_LR)]
        self.fp = FlatParams(spec, device, tail=2 * P)  # tail: a step's densification sums (gsr.dp)
        self.spatial_lr_scale = float(spatial_lr_scale)
        for name, v in (("xyz", xyz[~m]), ("scaling", scaling_raw), ("rotation", rotation_raw),
                        ("opacity", opacity_raw), ("albedo", albedo_raw), ("roughness", rough_raw),
                        ("metalness", metal_raw), ("sky_radius", torch.tensor([float(sky_radius)])),
                        ("sky_angles", cartesian_to_polar_coord(sky_pts, self.sky_center, float(sky_radius)))):
            self.fp.load(name, v)
        g = torch.Generator().manual_seed(seed)
        # embeddings: unit rows, as initialize_embeddings normalises its encoder's outputs
        self.fp.load("embeddings", F.normalize(torch.randn(n_views, EMBEDDING_DIM, generator=g), dim=-1))
        for name, fout, fin in MLP_LAYERS:  # nn.Linear's default: U(-1/sqrt(in), 1/sqrt(in))
            bound = 1.0 / math.sqrt(fin)
            self.fp.load(f"mlp.{name}.weight", (torch.rand(fout, fin, generator=g) * 2 - 1) * bound)
            self.fp.load(f"mlp.{name}.bias", (torch.rand(fout, generator=g) * 2 - 1) * bound)
        # one device generator for the iteration's random draws (dropout, SH noise, directions)
        self.rng = torch.Generator(device=device)
        self.rng.manual_seed(seed + 12345)
        self.id_cache = {}
        self.global_groups = {"embeddings"} | {n for n in self.fp.names if n.startswith("mlp.")} | set(SCENE_GROUPS)
        self.sky_center = self.sky_center.to(device)
        self.set_sky_flags(m.to(device))
        self.stats = {"xyz_gradient_accum": torch.zeros(P, 1, device=device),
                      "denom": torch.zeros(P, 1, device=device),
                      "max_radii2D": torch.zeros(P, device=device)}
        self.step_stats = None
        self.iteration = 0  # the reference's loop counter of the last step (train.py:55)

    def set_sky_flags(self, is_sky: torch.Tensor) -> None:
        self.is_sky = is_sky.reshape(-1, 1).bool()
        self.layout = SkyLayout(self.is_sky)
        self.P = self.layout.P

    @property
    def sky_radius(self) -> torch.Tensor:
        return self.fp.params["sky_radius"]

    def get_xyz(self, params=None) -> torch.Tensor:
        """gaussian_model.py:84-93 on the flat parameters (or on ``params``, a dict of leaves
        with the same names)."""
        p = self.fp.params if params is None else params
        sky = None
        if self.layout.n_sky:
            sky = sky_xyz(p["sky_angles"], p["sky_radius"], self.sky_center)
        return self.layout.xyz(p["xyz"], sky)

    def model_fused(self):
        """model() on the fused activation kernels (gsr_activations_*): one launch forward,
        and a backward that writes the raw parameters' gradients straight into the flat
        gradient (no per-leaf autograd accumulation).  GPU scenes only."""
        from .sink import GradSink
        p = self.fp.params
        box = [None]
        outs = _Activations.apply(self, box, p["xyz"], p["sky_angles"], p["sky_radius"], p["scaling"], p["rotation"],
                                  p["opacity"], p["albedo"], p["roughness"], p["metalness"])
        xyz, scaling, rotation, opacity, albedo, rough, metal = outs
        # the views' backward kernels add their gradients of these into one buffer each
        # (gsr.sink); _Activations.backward reads them
        box[0] = GradSink(dict(zip(_Activations.KEYS, outs)))
        return types.SimpleNamespace(get_xyz=xyz, get_scaling=scaling, get_rotation=rotation, get_opacity=opacity,
                                     get_albedo=albedo, get_roughness=rough, get_metalness=metal,
                                     get_is_sky=self.is_sky)

    def model(self, params=None):
        p = self.fp.params if params is None else params
        # get_xyz is made on the current (main) stream: the views render on side streams, and
        # a leaf consumed there would accumulate its gradient off the stream it lives on
        # (autograd's AccumulateGrad stream-mismatch warning)
        return types.SimpleNamespace(get_xyz=self.get_xyz(p), get_scaling=torch.exp(p["scaling"]),
                                     get_rotation=F.normalize(p["rotation"]), get_opacity=torch.sigmoid(p["opacity"]),
                                     get_albedo=torch.sigmoid(p["albedo"]), get_roughness=torch.sigmoid(p["roughness"]),
                                     get_metalness=torch.sigmoid(p["metalness"]), get_is_sky=self.is_sky)


_BLACK = {}


def train_step(scene: RelitScene, views: List, view_ids: List[int], gts: List[torch.Tensor], group=None,
               world: int = 1, bg=None, streams=None, rand: Dict[str, torch.Tensor] = None,
               iteration: int = None, render_fn=None, optimizer_step: bool = True) -> torch.Tensor:
    """One data-parallel iteration: this rank's views rendered and back-propagated, one
    all-reduce of the flat gradient, the densification statistics reduced, one fused Adam
    step with the mean gradient over all ranks' views.  ``streams``: HIP streams the views
    alternate over (None: the current stream).  The views are independent until the
    optimizer step, so one view's latency-bound geometry passes overlap another's tile
    passes; autograd runs each view's backward on its forward's stream.  ``rand``: the
    iteration's random draws (draw_step_randomness; default: from the scene's generator).
    ``iteration``: the reference's loop counter (default: the scene's last + 1), which
    switches the normal term on past reg_normal_from_iter and the sky-depth term past
    reg_sky_gauss_depth_from_iter.  Returns this rank's summed loss as a device scalar (no
    host synchronisation inside the step).  ``render_fn``: render()'s implementation (default
    the fused gsr.relit.render; gsr.relit.render_calls is render()'s own call sequence).
    ``optimizer_step=False`` stops after the gradient exchange (fp.grad holds the summed
    gradient; tests).

    Per view (train.py:66-120): envlight_sh, sky_sh = MLPNet(embedding); render() with
    envlight_sh + noise; loss = reconstruction + sky-BRDF (+ 0.05 normal once iteration >
    15000) (view_loss) + envl_sh_loss(envlight_sh) + 100 min_scale_loss(radii)
    (+ 0.05 depth_loss_gaussians once iteration > 0)."""
    import relit_shade

    from . import relit
    from . import dp as gdp
    fp = scene.fp
    dev = fp.device
    # the fused activations' backward overwrites the _ACT_OVERWRITES segments (a prefix of the
    # buffer), so only the rest is zeroed here (sky_radius included: the backward writes it
    # only when sky Gaussians exist); act_grads_written confirms the overwrite before Adam
    keep = _ACT_OVERWRITES if dev.type == "cuda" else ()
    fp.zero_grad(keep=keep)
    scene.act_grads_written = False
    scene.iteration = it = scene.iteration + 1 if iteration is None else int(iteration)
    lam_normal = LAMBDA_NORMAL if (it > REG_NORMAL_FROM_ITER and LAMBDA_NORMAL > 0) else 0.0
    if bg is None:  # one tensor per device: render()'s grey-background check is cached on it
        bg = _BLACK.get(str(dev))
        if bg is None:
            bg = _BLACK[str(dev)] = torch.zeros(3, device=dev)
    pipe = types.SimpleNamespace(compute_cov3D_python=False)
    main = torch.cuda.current_stream(dev)
    streams = [main] if not streams else list(streams)
    # the activations are computed once per iteration and the views' losses share one
    # backward (autograd sums the views' gradients exactly as sequential backwards would)
    pc = scene.model_fused() if dev.type == "cuda" else scene.model()
    # the environment MLP runs once for the rank's views, on the main stream (its leaves live
    # there): embeddings -> MLPNet (training-mode dropout) -> env SH (+ noise) and sky SH
    V = len(views)
    if rand is None:
        rand = draw_step_randomness(V, dev, scene.rng)
    key = tuple(int(v) for v in view_ids)
    ids = scene.id_cache.get(key)
    if ids is None:  # one host-to-device copy per view set, not per iteration
        ids = scene.id_cache[key] = torch.as_tensor(key, device=dev, dtype=torch.long)
    # index_select: its backward is one index_add (indexing's is a sort-based index_put, ~25 us)
    env_sh, sky_sh = mlp_forward(fp.params, torch.index_select(fp.params["embeddings"], 0, ids), rand["dropout"])
    # one view of each per-view row (unbind: one stacking kernel in the backward, where
    # indexing gives a zero tensor + copy per view)
    env_lit = (env_sh + rand["noise"]).unbind(0)
    sky_rows = sky_sh.unbind(0)
    losses, outs = [], []
    for i, (view, gt) in enumerate(zip(views, gts)):
        s = streams[i % len(streams)]
        s.wait_stream(main)
        with torch.cuda.stream(s):
            light = relit_shade.EnvironmentLight(env_lit[i], sh_degree=4)
            out = (render_fn or relit.render)(view, pc, light, sky_rows[i][None], 1, pipe, bg, debug=False)
            losses.append(view_loss(out, gt, view.sky_mask, view.occluders_mask, LAMBDA_DSSIM, LAMBDA_SKY_BRDF,
                                    lam_normal))
        outs.append(out)
    for s in streams:
        main.wait_stream(s)
    for t in losses:
        t.record_stream(main)
    # envlight, min-scale and sky-depth regularisers of every view at once, on the main stream
    radii = [o["radii"] for o in outs]
    for r in radii:
        r.record_stream(main)
    vms = torch.stack([v.world_view_transform for v in views]).float()
    reg = view_regularisers(pc, radii, vms, env_sh, rand["dirs"], depth_on=it > REG_SKY_GAUSS_DEPTH_FROM_ITER)
    total = torch.stack(losses).sum() + reg.sum()
    total.backward()
    for s in streams:
        main.wait_stream(s)
    for out in outs:
        out["viewspace_points"].grad.record_stream(main)
    if keep and not scene.act_grads_written:  # the activations' backward did not run: no stale values
        for n in keep:
            fp.params[n].grad.zero_()
    fp.check_grads_in_place()
    # densification statistics (train.py:130, 143-144), the iteration's one exchange and the
    # Adam step: at N > 1 the bucket's all-reduce goes out in chunks and each chunk's update
    # runs as soon as that chunk lands (gsr.dp.finish_step), so the update overlaps the exchange
    on_chunk = None
    if optimizer_step:
        apply_lr_schedule(scene, it)
        fp.begin_step(grad_scale=1.0 / (len(views) * max(world, 1)))
        on_chunk = fp.step_range
    gdp.finish_step(scene, [o["viewspace_points"].grad for o in outs], radii, it, world=world, group=group,
                    on_chunk=on_chunk)
    del outs
    return total.detach()


def synthetic_relit_scene(P_fg, n_views, W, H, focal, device, seed=0, sky_frac=0.1):
    """A cfg2-distributed relightable scene (z ~ logU(1, 30), screen radius
    ~10-20 px) with ``P_fg`` foreground + ``sky_frac * P_fg`` sky Gaussians, materials
    ~ U(0, 1), and ``n_views`` cameras jittered around the origin looking down +z (each with
    a sky mask over the top fifth of the frame, no occluders, and a fixed random target
    image).  Returns (RelitScene, views, gts)."""
    from . import scenes
    P = P_fg + int(P_fg * sky_frac)
    cam0 = scenes.focal_camera(W, H, focal)
    gs = scenes.synthetic_gaussians(P, W, H, cam0.tanfovx, cam0.tanfovy, 0, seed=seed, zrange=(1.0, 30.0),
                                    log_z=True, scale_mode="cfg2")
    g = torch.Generator().manual_seed(seed + 1)
    is_sky = torch.zeros(P, dtype=torch.bool)
    is_sky[P_fg:] = True
    # the sky Gaussians on a shell of radius 30 (the far end of the depth range) around the
    # origin, in the upper half of the frustum (COLMAP axes: -y is up), at the screen size
    # they were drawn with
    xyz, scales = gs["means3D"].clone(), gs["scales"].clone()
    d = xyz[P_fg:].clone()
    d[:, 1] = -d[:, 1].abs()
    r = d.norm(dim=1, keepdim=True)
    xyz[P_fg:] = 30.0 * d / r
    scales[P_fg:] *= 30.0 / r
    logit = lambda x: torch.log(x / (1 - x))
    scene = RelitScene(xyz, torch.log(scales), gs["rotations"], logit(gs["opacities"]),
                       logit(torch.rand(P_fg, 3, generator=g) * 0.9 + 0.05),
                       logit(torch.rand(P_fg, 1, generator=g) * 0.9 + 0.05),
                       logit(torch.rand(P_fg, 1, generator=g) * 0.9 + 0.05), is_sky, n_views, device, seed=seed,
                       sky_radius=30.0)
    views, gts = [], []
    for v in range(n_views):
        pos = (torch.rand(3, generator=g) - 0.5).numpy() * 0.4
        R, T = scenes.look_at_rotation(pos, [0.0, 0.0, 10.0])
        cam = scenes.focal_camera(W, H, focal, R=R, T=T, device=device)
        sky = torch.ones(1, H, W, device=device)
        sky[:, : H // 5] = 0.0
        views.append(types.SimpleNamespace(
            image_width=W, image_height=H, FoVx=cam.FoVx, FoVy=cam.FoVy,
            world_view_transform=cam.world_view_transform, full_proj_transform=cam.full_proj_transform,
            camera_center=cam.camera_center, sky_mask=sky, occluders_mask=torch.ones(1, H, W, device=device)))
        gts.append(torch.rand(3, H, W, generator=g).to(device))
    return scene, views, gts
