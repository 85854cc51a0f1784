"""densify_and_prune on the flat-parameter scene (gsr.train.RelitScene), rank-consistent
under view-parallel data parallelism.

Follows scene/gaussian_model.py:
  densify_and_prune   :610-625  grads = accum / denom (NaN -> 0); clone; split; prune on
                                opacity < min_opacity, and with max_screen_size also on
                                max_radii2D > max_screen_size or max scale > 0.1 extent
  densify_and_clone   :584-607  |grad| >= max_grad and max scale <= percent_dense * extent
  densify_and_split   :545-581  grad >= max_grad (padded over the clones) and max scale
                                > percent_dense * extent; N samples ~ normal(0, scale)
                                rotated by build_rotation(raw rotation) around the parent;
                                scale / (0.8 N); sky samples projected onto the sky shell;
                                parents pruned
  densification_postfix :514-542 appends rows; Adam moments of new rows are zero
                                (cat_tensors_to_optimizer :488-511); statistics reset
  prune_points        :465-485  rows removed from every group and from the Adam moments
                                (_prune_optimizer :438-462)

Per-Gaussian groups hold P rows (scaling, rotation, opacity), one row per foreground
Gaussian in foreground order (xyz, albedo, roughness, metalness) or one row per sky Gaussian
in sky order (sky_angles), as the reference's groups (_prune_optimizer :438-462).  A split
sky sample is projected onto the shell and turned back into angles with
cartesian_to_polar_coord's default radius of 1 (:571-573, as the reference calls it).

Rank consistency: every input of the decisions (parameters, reduced statistics) is
identical on every rank by construction, and the split's samples come from ``generator``,
which gsr.dp.shared_generator seeds identically on every rank.  So every rank performs the
same surgery and ends with bit-identical parameters and Adam state
(tests/test_dp_gloo.py::test_densify_rank_consistent).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from .train import FG_ROW_GROUPS as FG_GROUPS
from .train import SKY_ROW_GROUPS as SKY_GROUPS
from .train import FlatParams, SkyLayout, cartesian_to_polar_coord, sky_xyz


def build_rotation(r: torch.Tensor) -> torch.Tensor:
    """utils/general_utils.py build_rotation: normalised quaternion (w, x, y, z) -> R [N,3,3]."""
    q = r / torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])[:, None]
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.zeros((q.size(0), 3, 3), dtype=q.dtype, device=q.device)
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - w * z)
    R[:, 0, 2] = 2 * (x * z + w * y)
    R[:, 1, 0] = 2 * (x * y + w * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - w * x)
    R[:, 2, 0] = 2 * (x * z - w * y)
    R[:, 2, 1] = 2 * (y * z + w * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


class _Rows:
    """The scene's per-Gaussian groups as plain row tensors (value, exp_avg, exp_avg_sq)
    during the surgery; written back into a rebuilt FlatParams at the end."""

    def __init__(self, scene):
        fp = scene.fp
        self.t = {}
        for name, shape, off in zip(fp.names, fp.shapes, fp.offsets):
            n = 1
            for d in shape:
                n *= d
            self.t[name] = [buf[off:off + n].view(shape).clone() for buf in (fp.flat.detach(), fp.exp_avg,
                                                                           fp.exp_avg_sq)]
        self.is_sky = scene.is_sky.reshape(-1).clone()
        self.global_groups = scene.global_groups

    def get(self, name):
        return self.t[name][0]

    def append(self, new: Dict[str, torch.Tensor], new_is_sky: torch.Tensor) -> None:
        for name, v in new.items():
            val, m, s = self.t[name]
            self.t[name] = [torch.cat([val, v]), torch.cat([m, torch.zeros_like(v)]), torch.cat([s, torch.zeros_like(v)])]
        self.is_sky = torch.cat([self.is_sky, new_is_sky])

    def keep(self, mask: torch.Tensor) -> None:
        fg_mask, sky_mask = mask[~self.is_sky], mask[self.is_sky]
        for name in self.t:
            if name in self.global_groups:  # embeddings, MLP weights, sky radius: not per Gaussian
                continue
            m = fg_mask if name in FG_GROUPS else sky_mask if name in SKY_GROUPS else mask
            self.t[name] = [x[m] for x in self.t[name]]
        self.is_sky = self.is_sky[mask]

    def xyz(self, center: torch.Tensor) -> torch.Tensor:
        """get_xyz of the current rows (gaussian_model.py:84-93)."""
        sky = sky_xyz(self.get("sky_angles"), self.get("sky_radius"), center) if bool(self.is_sky.any()) else None
        return SkyLayout(self.is_sky).xyz(self.get("xyz"), sky)


def _reset_stats(scene, P, dev):
    scene.stats = {"xyz_gradient_accum": torch.zeros(P, 1, device=dev), "denom": torch.zeros(P, 1, device=dev),
                   "max_radii2D": torch.zeros(P, device=dev)}


def densify_and_prune(scene, max_grad: float, min_opacity: float, extent: float, max_screen_size: Optional[float],
                      percent_dense: float = 0.01, N: int = 2, generator: Optional[torch.Generator] = None,
                      group=None) -> None:
    """gaussian_model.py:610-625 on a RelitScene, in place (the scene's FlatParams is
    rebuilt with the new row counts; the Adam step count is kept).  Under data parallelism
    the ranks' rank-local max_radii2D (gsr.dp.finish_step) are MAX-reduced first: every rank
    must call this at the same iteration, as train.py's densification interval does."""
    if getattr(scene, "max_radii_local", False):
        from . import dp
        dp.sync_max_radii(scene.stats, group)
        scene.max_radii_local = False
    fp = scene.fp
    dev = fp.device
    rows = _Rows(scene)
    st = scene.stats
    with torch.no_grad():
        grads = st["xyz_gradient_accum"] / st["denom"]
        grads[grads.isnan()] = 0.0
        # ---- densify_and_clone (:584-607)
        scaling = torch.exp(rows.get("scaling"))
        sel = (torch.norm(grads, dim=-1) >= max_grad) & (scaling.max(dim=1).values <= percent_dense * extent)
        if bool(sel.any()):
            sel_fg, sel_sky = sel[~rows.is_sky], sel[rows.is_sky]
            new = {"scaling": rows.get("scaling")[sel], "rotation": rows.get("rotation")[sel],
                   "opacity": rows.get("opacity")[sel], "sky_angles": rows.get("sky_angles")[sel_sky]}
            new.update({g: rows.get(g)[sel_fg] for g in FG_GROUPS})
            rows.append(new, rows.is_sky[sel])
            # densification_postfix resets the statistics (:540-542)
            _reset_stats(scene, rows.is_sky.shape[0], dev)
        # ---- densify_and_split (:545-581)
        n_init = rows.is_sky.shape[0]
        padded = torch.zeros(n_init, device=dev)
        padded[:grads.shape[0]] = grads.squeeze()
        scaling = torch.exp(rows.get("scaling"))
        sel = (padded >= max_grad) & (scaling.max(dim=1).values > percent_dense * extent)
        if bool(sel.any()):
            sel_fg = sel[~rows.is_sky]
            stds = scaling[sel].repeat(N, 1)
            samples = torch.normal(mean=torch.zeros_like(stds), std=stds, generator=generator)
            rots = build_rotation(rows.get("rotation")[sel]).repeat(N, 1, 1)
            new_xyz = torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + rows.xyz(scene.sky_center)[sel].repeat(N, 1)
            new_sky = rows.is_sky[sel].repeat(N)
            new = {"scaling": torch.log(scaling[sel].repeat(N, 1) / (0.8 * N)),
                   "rotation": rows.get("rotation")[sel].repeat(N, 1), "opacity": rows.get("opacity")[sel].repeat(N, 1)}
            if bool(new_sky.any()):
                c = scene.sky_center
                d = new_xyz[new_sky] - c
                new_xyz[new_sky] = c + rows.get("sky_radius") * d / torch.norm(d, dim=1)[..., None]
                new["sky_angles"] = cartesian_to_polar_coord(new_xyz[new_sky], c)
            new["xyz"] = new_xyz[~new_sky]
            new.update({g: rows.get(g)[sel_fg].repeat(N, 1) for g in FG_GROUPS if g != "xyz"})
            rows.append(new, new_sky)
            _reset_stats(scene, rows.is_sky.shape[0], dev)
            prune = torch.cat([sel, torch.zeros(N * int(sel.sum()), device=dev, dtype=torch.bool)])
            rows.keep(~prune)
            scene.stats = {k: v[~prune] for k, v in scene.stats.items()}
        # ---- prune (:617-623)
        prune = (torch.sigmoid(rows.get("opacity")) < min_opacity).squeeze(1)
        if max_screen_size:
            big_vs = scene.stats["max_radii2D"] > max_screen_size
            big_ws = torch.exp(rows.get("scaling")).max(dim=1).values > 0.1 * extent
            prune = prune | big_vs | big_ws
        rows.keep(~prune)
        scene.stats = {k: v[~prune] for k, v in scene.stats.items()}
    _rebuild(scene, rows)


def _rebuild(scene, rows: _Rows) -> None:
    old = scene.fp
    spec = [(name, tuple(rows.t[name][0].shape), lr) for name, lr in zip(old.names, old.lrs)]
    fp = FlatParams(spec, old.device, betas=old.betas, eps=old.eps, tail=2 * rows.is_sky.shape[0])
    fp.t = old.t
    with torch.no_grad():
        for name, off in zip(fp.names, fp.offsets):
            val, m, s = rows.t[name]
            n = val.numel()
            fp.flat[off:off + n].copy_(val.reshape(-1))
            fp.exp_avg[off:off + n].copy_(m.reshape(-1))
            fp.exp_avg_sq[off:off + n].copy_(s.reshape(-1))
    scene.fp = fp
    scene.set_sky_flags(rows.is_sky)
    scene.step_stats = None
