"""Golden vectors for the training iteration's non-rasterizer pieces (train.py:66-120), made
by importing the REFERENCE's own Python (read-only at /root/reference) on the CPU with the
stubs of tools/gen_golden.py.  Output: tests/golden/train_step.npz (inputs + expected
outputs and gradients only; no reference source is stored).

    python tools/gen_golden_train.py

Pinned by these fixtures:
  MLPNet.forward          scene/net_models.py:16-52 (eval mode: dropout is the identity;
                          the train-mode mask is drawn explicitly by gsr.train) + autograd
                          gradients of every weight and of the embedding
  envl_sh_loss            utils/loss_utils.py:185-207 (the 10 random directions are redrawn
                          from the same seeded CPU generator and stored)
  min_scale_loss          utils/loss_utils.py:210-220
  depth_loss_gaussians    utils/loss_utils.py:140-148 (+ GaussianModel.get_depth :125-130)
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


if __name__ == "__main__":
    main()
