"""Golden vectors for the training iteration's non-rasterizer pieces (train.py:66-120), made
by importing the REFERENCE's own Python (read-only at /root/reference) on the CPU with the
stubs of tools/gen_golden.py.  Output: tests/golden/train_step.npz (inputs + expected
outputs and gradients only; no reference source is stored).

    python tools/gen_golden_train.py        (everything)
    python tools/gen_golden_train.py lr     (tests/golden/train_lr.npz only)
    python tools/gen_golden_train.py iteration   (tests/golden/train_iter.npz only)

Pinned by these fixtures:
  MLPNet.forward          scene/net_models.py:16-52 (eval mode: dropout is the identity;
                          the train-mode mask is drawn explicitly by gsr.train) + autograd
                          gradients of every weight and of the embedding
  envl_sh_loss            utils/loss_utils.py:185-207 (the 10 random directions are redrawn
                          from the same seeded CPU generator and stored)
  min_scale_loss          utils/loss_utils.py:210-220
  depth_loss_gaussians    utils/loss_utils.py:140-148 (+ GaussianModel.get_depth :125-130)

and tests/golden/train_sky.npz:
  get_xyz / get_sky_xyz / get_sky_angles   scene/gaussian_model.py:84-103,159-169 (sky
                          Gaussians as clamped (theta, phi) on a shell of learnable radius,
                          interleaved with the foreground rows) + autograd gradients
  cartesian_to_polar_coord utils/general_utils.py:295-299 (default and explicit radius)
  densify_and_prune       scene/gaussian_model.py:438-625 on a GaussianModel with an Adam
                          state (one torch.optim.Adam step first): clone, split (sky samples
                          projected onto the shell, angles back with the default radius),
                          prune; every group's rows and moments before and after, under a
                          fixed torch.manual_seed for the split's torch.normal
"""
import os
import sys
import types

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_golden  # noqa: E402

OUT = gen_golden.OUT


def main():
    gen_golden.setup_reference_import()
    gen_golden._stub("data")
    gen_golden._stub("data.dataloader_net", load_train_test=None)
    sys.modules["data"].dataloader_net = sys.modules["data.dataloader_net"]
    from scene.gaussian_model import GaussianModel
    from scene.net_models import MLPNet
    from utils import loss_utils

    rng = np.random.default_rng(4321)
    fx = {}

    # ---------------- MLPNet (embedding -> env SH deg 4 + sky SH deg 1) ------------------
    torch.manual_seed(7)
    net = MLPNet(sh_degree_envl=4, sh_degree_sky=1, embedding_dim=32)
    net.eval()
    B = 5
    e = torch.tensor(rng.normal(0, 1, (B, 32)), dtype=torch.float32)
    e = (e / e.norm(dim=1, keepdim=True)).requires_grad_(True)
    env, sky = net(e)
    g_env = torch.tensor(rng.normal(0, 1, tuple(env.shape)), dtype=torch.float32)
    g_sky = torch.tensor(rng.normal(0, 1, tuple(sky.shape)), dtype=torch.float32)
    names = [n for n, _ in net.named_parameters()]
    grads = torch.autograd.grad([env, sky], [e] + list(net.parameters()), [g_env, g_sky])
    fx["mlp/emb"] = e.detach().numpy()
    fx["mlp/env"] = env.detach().numpy()
    fx["mlp/sky"] = sky.detach().numpy()
    fx["mlp/g_env"] = g_env.numpy()
    fx["mlp/g_sky"] = g_sky.numpy()
    fx["mlp/d_emb"] = grads[0].numpy()
    fx["mlp/param_names"] = np.array(names)
    for n, p, g in zip(names, net.parameters(), grads[1:]):
        fx[f"mlp/w/{n}"] = p.detach().numpy()
        fx[f"mlp/dw/{n}"] = g.numpy()

    # ---------------- envl_sh_loss --------------------------------------------------------
    for ci, scale in enumerate((0.3, 1.5)):
        sh = torch.tensor(rng.normal(0, scale, (1, 25, 3)), dtype=torch.float32)
        sh[0, 0] = 0.2
        sh = sh.requires_grad_(True)
        torch.manual_seed(100 + ci)
        loss = loss_utils.envl_sh_loss(sh, 4)
        loss = loss if torch.is_tensor(loss) else torch.tensor(float(loss))
        (d_sh,) = torch.autograd.grad(loss, [sh], allow_unused=True) if loss.requires_grad else (None,)
        torch.manual_seed(100 + ci)  # the same draw envl_sh_loss made (utils/loss_utils.py:188)
        dirs = torch.empty(10, 3).uniform_(-1, 1)
        fx[f"envl{ci}/sh"] = sh.detach().numpy()
        fx[f"envl{ci}/dirs_unnorm"] = dirs.numpy()
        fx[f"envl{ci}/loss"] = np.array(float(loss), np.float32)
        fx[f"envl{ci}/d_sh"] = np.zeros_like(sh.detach().numpy()) if d_sh is None else d_sh.numpy()

    # ---------------- min_scale_loss and depth_loss_gaussians ---------------------------
    P = 300
    is_sky = torch.zeros(P, 1, dtype=torch.bool)
    is_sky[rng.choice(P, 60, replace=False)] = True
    radii = torch.tensor(rng.integers(0, 3, P), dtype=torch.int32)  # ~1/3 culled
    scaling = torch.tensor(np.exp(rng.normal(np.log(0.05), 0.6, (P, 3))), dtype=torch.float32).requires_grad_(True)
    xyz = torch.tensor(rng.normal(0, 2, (P, 3)) + np.array([0.0, 0.0, 8.0]), dtype=torch.float32)
    xyz[is_sky.squeeze()] *= 4.0
    xyz = xyz.requires_grad_(True)
    a = rng.normal(0, 0.2, 3)
    th = np.linalg.norm(a)
    k = a / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    Rm = np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx
    from utils import graphics_utils as gfx
    wvt = torch.tensor(gfx.getWorld2View2(Rm, rng.normal(0, 0.5, 3))).transpose(0, 1).float()
    gs = types.SimpleNamespace(get_scaling=scaling, get_is_sky=is_sky, get_xyz=xyz)
    gs.get_depth = types.MethodType(GaussianModel.get_depth, gs)
    cam = types.SimpleNamespace(world_view_transform=wvt)
    ms = loss_utils.min_scale_loss(radii, gs)
    (d_scaling,) = torch.autograd.grad(ms, [scaling])
    vis = radii > 0
    dl = loss_utils.depth_loss_gaussians(gs, cam, vis)
    (d_xyz,) = torch.autograd.grad(dl, [xyz])
    fx.update({"reg/is_sky": is_sky.numpy(), "reg/radii": radii.numpy(), "reg/scaling": scaling.detach().numpy(),
               "reg/xyz": xyz.detach().numpy(), "reg/viewmatrix": wvt.numpy(),
               "reg/min_scale_loss": np.array(float(ms), np.float32), "reg/d_scaling": d_scaling.numpy(),
               "reg/depth_loss": np.array(float(dl), np.float32), "reg/d_xyz": d_xyz.numpy()})
    np.savez_compressed(os.path.join(OUT, "train_step.npz"), **fx)
    print("wrote", os.path.join(OUT, "train_step.npz"))
    sky_and_densify(GaussianModel)


GROUPS = ("xyz", "albedo", "opacity", "scaling", "rotation", "roughness", "metalness", "sky_radius", "sky_angles")


def sky_and_densify(GaussianModel):
    from torch import nn

    from utils import general_utils as gu
    rng = np.random.default_rng(777)
    fx = {}
    t = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32)

    # ---------------- get_xyz with sky angles (interleaved rows, out-of-range angles) -----
    P, n_sky = 240, 60
    is_sky = np.zeros((P, 1), bool)
    is_sky[rng.choice(P, n_sky, replace=False)] = True
    gm = GaussianModel()
    gm._xyz = nn.Parameter(t(rng.normal(0, 2, (P - n_sky, 3))))
    ang = np.stack([rng.uniform(-0.3, np.pi / 2 + 0.3, n_sky), rng.uniform(-np.pi / 2 - 0.3, np.pi / 2 + 0.3, n_sky)], 1)
    gm._sky_angles = nn.Parameter(t(ang))
    gm._sky_radius = nn.Parameter(torch.tensor(7.5))
    gm._sky_gauss_center = t([[0.3, -0.2, 1.0]])
    gm._is_sky = torch.tensor(is_sky)
    xyz = gm.get_xyz
    g = t(rng.normal(0, 1, (P, 3)))
    d_xyz, d_ang, d_rad = torch.autograd.grad(xyz, [gm._xyz, gm._sky_angles, gm._sky_radius], g)
    fx.update({"sky/is_sky": is_sky, "sky/xyz_fg": gm._xyz.detach().numpy(), "sky/angles": ang.astype(np.float32),
               "sky/radius": np.float32(7.5), "sky/center": np.float32([0.3, -0.2, 1.0]),
               "sky/get_xyz": xyz.detach().numpy(), "sky/g": g.numpy(), "sky/d_xyz_fg": d_xyz.numpy(),
               "sky/d_angles": d_ang.numpy(), "sky/d_radius": np.float32(d_rad)})
    pts = t(rng.normal(0, 5, (50, 3)))
    c = t([0.3, -0.2, 1.0])
    fx["c2p/pts"] = pts.numpy()
    fx["c2p/center"] = c.numpy()
    fx["c2p/default_radius"] = gu.cartesian_to_polar_coord(pts, c).numpy()
    fx["c2p/radius_7_5"] = gu.cartesian_to_polar_coord(pts, c, 7.5).numpy()

    # ---------------- densify_and_prune with an Adam state ---------------------------------
    P, n_sky = 400, 80
    is_sky = np.zeros((P, 1), bool)
    is_sky[rng.choice(P, n_sky, replace=False)] = True
    n_fg = P - n_sky
    gm = GaussianModel()
    gm.percent_dense = 0.01
    center = t([[0.1, 0.0, 0.5]])
    radius = 6.0
    sky_dirs = rng.normal(0, 1, (n_sky, 3))
    sky_dirs[:, 1] = -np.abs(sky_dirs[:, 1])
    sky_dirs[:, 2] = np.abs(sky_dirs[:, 2])
    sky_pts = center + radius * t(sky_dirs / np.linalg.norm(sky_dirs, axis=1, keepdims=True))
    gm._xyz = nn.Parameter(t(rng.normal(0, 1.5, (n_fg, 3))))
    gm._sky_gauss_center = center
    gm._sky_radius = nn.Parameter(torch.tensor(radius))
    gm._sky_angles = nn.Parameter(gu.cartesian_to_polar_coord(sky_pts, center.squeeze(), gm._sky_radius).detach())
    # scales straddling percent_dense * extent (extent 4 -> 0.04): clones below, splits above
    gm._scaling = nn.Parameter(t(np.log(np.exp(rng.normal(np.log(0.04), 0.8, (P, 3))))))
    gm._rotation = nn.Parameter(t(rng.normal(0, 1, (P, 4))))
    gm._opacity = nn.Parameter(t(rng.normal(0, 2, (P, 1))))
    gm._albedo = nn.Parameter(t(rng.normal(0, 1, (n_fg, 3))))
    gm._roughness = nn.Parameter(t(rng.normal(0, 1, (n_fg, 1))))
    gm._metalness = nn.Parameter(t(rng.normal(0, 1, (n_fg, 1))))
    gm._is_sky = torch.tensor(is_sky)
    params = {n: getattr(gm, "_" + n) for n in GROUPS}
    lrs = {"xyz": 1e-3, "albedo": 2.5e-3, "opacity": 0.05, "scaling": 1e-3, "rotation": 1e-3, "roughness": 2e-4,
           "metalness": 2e-4, "sky_radius": 1e-4, "sky_angles": 1e-3}
    gm.optimizer = torch.optim.Adam([{"params": [params[n]], "lr": lrs[n], "name": n} for n in GROUPS], lr=0.0,
                                    eps=1e-15)
    for n in GROUPS:  # one step with fixed gradients: every group gets an Adam state
        params[n].grad = t(rng.normal(0, 1e-2, tuple(params[n].shape)))
    gm.optimizer.step()
    accum = np.abs(rng.normal(0, 1, (P, 1))) * 2e-4
    denom = rng.integers(0, 3, (P, 1)).astype(np.float32)
    gm.xyz_gradient_accum = t(accum)
    gm.denom = t(denom)
    gm.max_radii2D = t(rng.integers(0, 30, P))
    for n in GROUPS:
        st = gm.optimizer.state[params[n]]
        fx[f"dens/before/{n}"] = params[n].detach().numpy()
        fx[f"dens/before/m/{n}"] = st["exp_avg"].numpy()
        fx[f"dens/before/v/{n}"] = st["exp_avg_sq"].numpy()
    fx.update({"dens/before/is_sky": is_sky, "dens/center": center.numpy().reshape(3),
               "dens/accum": accum.astype(np.float32), "dens/denom": denom,
               "dens/max_radii2D": gm.max_radii2D.numpy(), "dens/seed": np.int64(2024),
               "dens/args": np.float32([1e-4, 0.1, 4.0, 20.0])})  # max_grad, min_opacity, extent, max_screen_size
    torch.manual_seed(2024)
    gm.densify_and_prune(1e-4, 0.1, 4.0, 20.0, None)
    for n in GROUPS:
        p = gm.optimizer.param_groups[[gr["name"] for gr in gm.optimizer.param_groups].index(n)]["params"][0]
        st = gm.optimizer.state[p]
        fx[f"dens/after/{n}"] = p.detach().numpy()
        fx[f"dens/after/m/{n}"] = st["exp_avg"].numpy()
        fx[f"dens/after/v/{n}"] = st["exp_avg_sq"].numpy()
    fx["dens/after/is_sky"] = gm._is_sky.numpy()
    fx["dens/after/get_xyz"] = gm.get_xyz.detach().numpy()
    np.savez_compressed(os.path.join(OUT, "train_sky.npz"), **fx)
    print("wrote", os.path.join(OUT, "train_sky.npz"), {k: v.shape for k, v in fx.items() if k.startswith("dens/a")})


LR_ITERS = (1, 2, 3, 100, 500, 14999, 15000, 15001, 15002, 19999, 20000, 20001, 20002, 29999, 30000, 30001, 30002,
            39999, 40000)


def lr_schedule():
    """tests/golden/train_lr.npz: the learning rate every param group's Adam step uses at the
    iterations LR_ITERS, from the reference's own training_setup groups, get_expon_lr_func
    (utils/general_utils.py:46-80) and update_learning_rate (gaussian_model.py:285-290 through
    relit3DGW_model.py:153-158), driven as train.py:156-159 drives them: step, then
    update_learning_rate(iteration).  Twice: the default config (mlp_lr = embeddings_lr =
    0.0002, so the iteration-20000 reset is a no-op) and mlp_lr = embeddings_lr = 0.001 (the
    reset visible), both with spatial_lr_scale 2.5."""
    gen_golden.setup_reference_import()
    gen_golden._stub("data")
    gen_golden._stub("data.dataloader_net", load_train_test=None)
    sys.modules["data"].dataloader_net = sys.modules["data.dataloader_net"]
    from scene.gaussian_model import GaussianModel
    from utils.general_utils import get_expon_lr_func
    # relit3DGW_model's module-level imports: hydra's decorator as the identity, the config and
    # dataset types as placeholders (only the unbound update_learning_rate is called)
    gen_golden._stub("omegaconf", OmegaConf=object, DictConfig=object)
    gen_golden._stub("hydra", main=lambda **kw: (lambda f: f))
    gen_golden._stub("torchvision")
    for m in ("diff_gaussian_rasterization",):
        if m not in sys.modules:
            gen_golden._stub(m, GaussianRasterizationSettings=object, GaussianRasterizer=object)
    sys.modules["scene"].GaussianModel = GaussianModel
    sys.modules["scene"].Scene = object
    from scene.relit3DGW_model import Relightable3DGW
    scale = 2.5
    fx = {"lr/iters": np.array(LR_ITERS), "lr/spatial_lr_scale": np.array(scale)}
    for tag, mlp_lr in (("default", 0.0002), ("mlp1e-3", 0.001)):
        lrs0 = {"xyz": 0.00016 * scale, "albedo": 0.0025, "opacity": 0.05, "scaling": 0.001 * scale,
                "rotation": 0.001, "roughness": 0.0002, "metalness": 0.0002, "sky_radius": 0.0001,
                "sky_angles": 0.00016 * scale, "mlp": mlp_lr, "embeddings": mlp_lr}
        groups = [{"params": [torch.zeros(1, requires_grad=True)], "lr": lr, "name": n} for n, lr in lrs0.items()]
        opt = torch.optim.Adam(groups, lr=0.01, eps=1e-15)
        gm = types.SimpleNamespace(optimizer=opt, xyz_scheduler_args=get_expon_lr_func(
            lr_init=0.00016 * scale, lr_final=0.0000016 * scale, lr_delay_mult=0.01, max_steps=30_000))
        gm.update_learning_rate = types.MethodType(GaussianModel.update_learning_rate, gm)
        model = types.SimpleNamespace(gaussians=gm, optimizer=opt)
        names = [g["name"] for g in opt.param_groups]
        rec = {n: [] for n in names}
        want = set(LR_ITERS)
        for it in range(1, max(LR_ITERS) + 1):
            if it in want:  # the rates this iteration's step uses
                for g in opt.param_groups:
                    rec[g["name"]].append(g["lr"])
            Relightable3DGW.update_learning_rate(model, it)
        for n in names:
            fx[f"lr/{tag}/{n}"] = np.array(rec[n], np.float64)
    np.savez_compressed(os.path.join(OUT, "train_lr.npz"), **fx)
    print("wrote", os.path.join(OUT, "train_lr.npz"))


def iteration():
    """tests/golden/train_iter.npz: ONE training iteration of the reference, composed as
    train.py:62-159 composes it from the reference's own pieces -- the embedding row through
    MLPNet (training-mode dropout, with the mask drawn here and stored), the environment SH
    plus N(0, 0.025) noise (stored) into EnvironmentLight.set_base, render() (debug=False,
    specular, fix_sky off; the C oracle stands in for diff_gaussian_rasterization, as in
    tools/gen_golden_render.py), the reconstruction (L1 + D-SSIM under the occluder mask),
    sky-BRDF, normal-consistency (iteration 15001 > reg_normal_from_iter), envlight (its random
    directions re-drawn from the same seed and stored), min-scale and sky-depth losses with the
    configured weights, loss.backward(), the Adam step over Relightable3DGW.training_set_up's
    groups (lr 0.01, eps 1e-15; every group with an Adam state from one earlier step with fixed
    gradients, so the step is not sign-dominated) and update_learning_rate(iteration).  The
    scene is a GaussianModel with interleaved sky Gaussians on their (theta, phi) shell.
    Stored: every raw parameter and Adam moment before, the step's raw gradients, the
    parameters after, the loss, and the inputs (camera, target, masks, draws)."""
    import yaml
    from torch import nn

    gen_golden.setup_reference_import()
    gen_golden._stub("data")
    gen_golden._stub("data.dataloader_net", load_train_test=None)
    sys.modules["data"].dataloader_net = sys.modules["data.dataloader_net"]
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import oracle_torch
    stub = types.ModuleType("diff_gaussian_rasterization")
    stub.GaussianRasterizationSettings = oracle_torch.GaussianRasterizationSettings
    stub.GaussianRasterizer = oracle_torch.GaussianRasterizer
    stub.rasterize_gaussians = oracle_torch.rasterize_gaussians
    sys.modules["diff_gaussian_rasterization"] = stub
    gen_golden._stub("omegaconf", OmegaConf=object, DictConfig=object)
    gen_golden._stub("hydra", main=lambda **kw: (lambda f: f))
    gen_golden._stub("torchvision")
    from scene.gaussian_model import GaussianModel
    sys.modules["scene"].GaussianModel = GaussianModel
    sys.modules["scene"].Scene = object
    from gaussian_renderer import render
    from scene.cameras import Camera
    from scene.NVDIFFREC.light import EnvironmentLight
    from scene.net_models import MLPNet
    from scene.relit3DGW_model import Relightable3DGW
    from utils import general_utils as gu
    from utils.loss_utils import depth_loss_gaussians, envl_sh_loss, l1_loss, min_scale_loss, ssim

    cfg = yaml.load(open(os.path.join(gen_golden.REF, "configs", "optimizer", "optimization_params.yaml")),
                    Loader=yaml.SafeLoader)
    top = yaml.load(open(os.path.join(gen_golden.REF, "configs", "relightable3DG-W.yaml")), Loader=yaml.SafeLoader)
    opt = types.SimpleNamespace(**cfg)
    rng = np.random.default_rng(31)
    torch.manual_seed(31)
    t = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32)
    W, H, P, n_sky, n_views, vid, iteration = 64, 48, 700, 70, 2, 1, 15001
    is_sky = np.zeros((P, 1), bool)
    is_sky[rng.choice(P, n_sky, replace=False)] = True
    n_fg = P - n_sky
    gm = GaussianModel()
    gm.spatial_lr_scale = 1.0
    center = t([[0.0, 0.0, 0.0]])
    radius = 30.0
    sky_dirs = rng.normal(0, 1, (n_sky, 3)) * [0.35, 0.25, 1.0]
    sky_dirs[:, 1] = -np.abs(sky_dirs[:, 1])
    sky_dirs[:, 2] = np.abs(sky_dirs[:, 2])
    sky_pts = center + radius * t(sky_dirs / np.linalg.norm(sky_dirs, axis=1, keepdims=True))
    gm._xyz = nn.Parameter(t(rng.normal(0, 1.0, (n_fg, 3)) * [1.2, 0.9, 1.0] + [0.0, 0.0, 5.0]))
    gm._sky_gauss_center = center
    gm._sky_radius = nn.Parameter(torch.tensor(radius))
    gm._sky_angles = nn.Parameter(gu.cartesian_to_polar_coord(sky_pts, center.squeeze(), gm._sky_radius).detach())
    sc = rng.normal(np.log(0.07), 0.4, (P, 3))
    sc[is_sky[:, 0]] += np.log(10.0)
    gm._scaling = nn.Parameter(t(sc))
    gm._rotation = nn.Parameter(t(rng.normal(0, 1, (P, 4))))
    gm._opacity = nn.Parameter(t(rng.normal(-0.5, 1.0, (P, 1))))
    gm._albedo = nn.Parameter(t(rng.normal(0, 1, (n_fg, 3))))
    gm._roughness = nn.Parameter(t(rng.normal(0, 1, (n_fg, 1))))
    gm._metalness = nn.Parameter(t(rng.normal(0, 1, (n_fg, 1))))
    gm._is_sky = torch.tensor(is_sky)
    gm.max_radii2D = torch.zeros(P)
    groups = gm.training_setup(opt)
    mlp = MLPNet(sh_degree_envl=top["envlight_sh_degree"], sh_degree_sky=top["sky_sh_degree"],
                 embedding_dim=top["embeddings_dim"])
    mlp.train()
    emb = nn.Embedding(n_views, top["embeddings_dim"])
    emb.weight = nn.Parameter(torch.nn.functional.normalize(t(rng.normal(0, 1, (n_views, top["embeddings_dim"]))),
                                                            p=2, dim=-1))
    params = [{"params": mlp.parameters(), "lr": opt.mlp_lr, "name": "mlp"},
              {"params": emb.parameters(), "lr": opt.embeddings_lr, "name": "embeddings"}] + groups
    optimizer = torch.optim.Adam(params, lr=0.01, eps=1e-15)  # relit3DGW_model.py:147-149
    gm.optimizer = optimizer
    named = {n: getattr(gm, "_" + n) for n in GROUPS}
    named.update({f"mlp.{n}": p for n, p in mlp.named_parameters()})
    named["embeddings"] = emb.weight
    # an earlier step with fixed gradients: every parameter has an Adam state
    for n, p in named.items():
        p.grad = t(rng.normal(0, 1e-2, tuple(p.shape)))
    optimizer.step()
    optimizer.zero_grad(set_to_none=True)
    fx = {"it/W": np.array(W), "it/H": np.array(H), "it/iteration": np.array(iteration), "it/vid": np.array(vid),
          "it/n_views": np.array(n_views), "it/is_sky": is_sky, "it/center": center.numpy().reshape(3),
          "it/names": np.array(list(named))}
    for n, p in named.items():
        st = optimizer.state[p]
        fx[f"before/{n}"] = p.detach().numpy().copy()
        fx[f"before/m/{n}"] = st["exp_avg"].numpy().copy()
        fx[f"before/v/{n}"] = st["exp_avg_sq"].numpy().copy()
        fx[f"before/step/{n}"] = np.array(float(st["step"]))

    # the camera (scene/cameras.py), its target, sky and occluder masks
    a = np.array([0.05, -0.08, 0.03])
    th = np.linalg.norm(a)
    k = a / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    Rm = np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx
    Tv = np.array([0.1, -0.05, 0.2])
    fovx = np.radians(60.0)
    fovy = 2 * np.arctan(np.tan(fovx / 2) * H / W)
    sky_mask = (rng.uniform(0, 1, (1, H, W)) > 0.25).astype(np.float32)
    occ_mask = (rng.uniform(0, 1, (1, H, W)) > 0.1).astype(np.float32)
    gt = rng.uniform(0, 1, (3, H, W)).astype(np.float32)
    cam = Camera(colmap_id=0, R=Rm, T=Tv, FoVx=fovx, FoVy=fovy, image=torch.from_numpy(gt), gt_alpha_mask=None,
                 image_name="iter", uid=vid, data_device="cpu", sky_mask=torch.from_numpy(sky_mask))
    cam.occluders_mask = torch.from_numpy(occ_mask)
    # the draws: MLPNet's dropout multiplier (0 or 1/(1-p), as nn.Dropout in training mode), the
    # environment SH noise, the envlight directions (envl_sh_loss's own draw, same seed)
    drop = (torch.rand(1, 256) >= 0.2).float() / 0.8

    class FixedDropout(nn.Module):
        def forward(self, x):
            return x * drop
    assert isinstance(mlp.base[1], nn.Dropout)
    mlp.base[1] = FixedDropout()
    noise = torch.randn(1, 25, 3) * 0.025

    # ---- train.py:62-118 ----
    viewpoint_cam_id = torch.tensor([vid])
    gt_image = cam.original_image
    sky_m = cam.sky_mask.expand_as(gt_image)
    occluders_mask = cam.occluders_mask.expand_as(gt_image)
    embedding_gt_image = emb(viewpoint_cam_id)
    envlight_sh, sky_sh = mlp(embedding_gt_image)
    envlight = EnvironmentLight(base=torch.zeros(25, 3), sh_degree=top["envlight_sh_degree"])
    envlight.set_base(envlight_sh + noise)
    pipe = types.SimpleNamespace(compute_cov3D_python=False)
    background = torch.zeros(3)
    render_pkg = render(cam, gm, envlight, sky_sh, top["sky_sh_degree"], pipe, background, debug=False,
                        fix_sky=top["fix_sky"], specular=top["specular"])
    image, radii = render_pkg["render"], render_pkg["radii"]
    visibility_filter = render_pkg["visibility_filter"]
    diff_col, spec_col = render_pkg["diffuse_color"], render_pkg["specular_color"]
    Ll1 = l1_loss(image, gt_image, mask=occluders_mask)
    Ssim = (1.0 - ssim(image, gt_image, mask=occluders_mask))
    loss = Ll1 * (1 - opt.lambda_dssim) + opt.lambda_dssim * Ssim
    loss_sky_brdf = l1_loss(diff_col, torch.zeros_like(diff_col), mask=1 - sky_m) + \
        l1_loss(spec_col, torch.zeros_like(spec_col), mask=1 - sky_m)
    loss = loss + opt.lambda_sky_brdf * loss_sky_brdf
    assert iteration > opt.reg_normal_from_iter and opt.lambda_normal > 0
    rendered_normal = render_pkg["normal"] * occluders_mask * sky_m
    rendered_surf_normal = render_pkg["normal_ref"] * occluders_mask * sky_m
    ncl = (1 - (rendered_normal * rendered_surf_normal).sum(dim=0))[None]
    loss = loss + opt.lambda_normal * ncl.mean()
    torch.manual_seed(4711)
    loss = loss + envl_sh_loss(envlight_sh, top["envlight_sh_degree"])
    torch.manual_seed(4711)
    dirs = torch.empty(10, 3).uniform_(-1, 1)  # the draw envl_sh_loss made (utils/loss_utils.py:188)
    loss = loss + opt.lambda_scale * min_scale_loss(radii, gm)
    assert iteration > opt.reg_sky_gauss_depth_from_iter and opt.lambda_sky_gauss > 0
    loss = loss + opt.lambda_sky_gauss * depth_loss_gaussians(gm, cam, visibility_filter)
    loss.backward()
    for n, p in named.items():
        fx[f"grad/{n}"] = p.grad.numpy().copy()
    # the rates this step uses: the loop called update_learning_rate(iteration - 1) at the end of
    # the previous iteration (train.py:159; training_setup made gm.xyz_scheduler_args)
    model = types.SimpleNamespace(gaussians=gm, optimizer=optimizer)
    Relightable3DGW.update_learning_rate(model, iteration - 1)
    fx["it/lrs"] = np.array([g["lr"] for g in optimizer.param_groups], np.float64)
    optimizer.step()  # train.py:156-159
    for n, p in named.items():
        fx[f"after/{n}"] = p.detach().numpy().copy()
    fx["after/lr_groups"] = np.array([g["name"] for g in optimizer.param_groups])
    fx["it/loss"] = np.array(float(loss.detach()), np.float64)
    fx["it/dropout"] = drop.numpy()
    fx["it/noise"] = noise.numpy()
    fx["it/dirs"] = dirs.numpy()
    fx["it/gt"] = gt
    fx["it/sky_mask"] = sky_mask
    fx["it/occ_mask"] = occ_mask
    fx["it/FoVx"] = np.array(fovx)
    fx["it/FoVy"] = np.array(fovy)
    fx["it/world_view_transform"] = cam.world_view_transform.numpy()
    fx["it/full_proj_transform"] = cam.full_proj_transform.numpy()
    fx["it/camera_center"] = cam.camera_center.numpy()
    fx["it/radii"] = radii.numpy()
    np.savez_compressed(os.path.join(OUT, "train_iter.npz"), **fx)
    print("wrote", os.path.join(OUT, "train_iter.npz"), "loss", float(loss), "visible", int((radii > 0).sum()))


if __name__ == "__main__":
    if sys.argv[1:] == ["lr"]:
        lr_schedule()
    elif sys.argv[1:] == ["iteration"]:
        iteration()
    else:
        main()
        lr_schedule()
        iteration()
