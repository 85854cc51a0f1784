"""CPU: the training iteration's non-rasterizer pieces in gsr.train against fixtures the
reference's own Python produced (tests/golden/train_step.npz, tools/gen_golden_train.py):
MLPNet forward + every gradient (scene/net_models.py:16-52), envl_sh_loss
(utils/loss_utils.py:185-207), min_scale_loss (:210-220) and depth_loss_gaussians (:140-148).
Tolerance: 1e-5 relative (fp32, different summation order)."""
import os
import types

import numpy as np
import pytest
import torch

from helpers import rel_l2

GOLD = os.path.join(os.path.dirname(__file__), "golden", "train_step.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def test_mlp_forward_and_gradients(gold):
    from gsr import train
    names = [str(n) for n in gold["mlp/param_names"]]
    assert names == [f"{l}.{k}" for l, _, _ in train.MLP_LAYERS for k in ("weight", "bias")]
    params = {f"mlp.{n}": torch.tensor(gold[f"mlp/w/{n}"]).requires_grad_(True) for n in names}
    for l, fout, fin in train.MLP_LAYERS:
        assert tuple(params[f"mlp.{l}.weight"].shape) == (fout, fin)
    e = torch.tensor(gold["mlp/emb"]).requires_grad_(True)
    env, sky = train.mlp_forward(params, e)
    assert rel_l2(env.detach().numpy(), gold["mlp/env"]) < 1e-6
    assert rel_l2(sky.detach().numpy(), gold["mlp/sky"]) < 1e-6
    grads = torch.autograd.grad([env, sky], [e] + [params[f"mlp.{n}"] for n in names],
                                [torch.tensor(gold["mlp/g_env"]), torch.tensor(gold["mlp/g_sky"])])
    assert rel_l2(grads[0].numpy(), gold["mlp/d_emb"]) < 1e-5
    for n, g in zip(names, grads[1:]):
        assert rel_l2(g.numpy(), gold[f"mlp/dw/{n}"]) < 1e-5, n


def test_mlp_dropout_is_inverted_scaling():
    """Training-mode dropout after the first layer (Linear -> Dropout -> ReLU): the mask
    multiplies the first layer's output by 0 or 1/(1-p) before the ReLU."""
    from gsr import train
    g = torch.Generator().manual_seed(0)
    params = {}
    for l, fout, fin in train.MLP_LAYERS:
        params[f"mlp.{l}.weight"] = torch.randn(fout, fin, generator=g) * 0.1
        params[f"mlp.{l}.bias"] = torch.randn(fout, generator=g) * 0.1
    e = torch.randn(3, 32, generator=g)
    rnd = train.draw_step_randomness(3, "cpu", g)
    m = rnd["dropout"]
    assert set(torch.unique(m).tolist()) <= {0.0, 1.0 / 0.8}
    assert 0.1 < float((m == 0).float().mean()) < 0.3
    env, sky = train.mlp_forward(params, e, m)
    h = torch.relu(torch.nn.functional.linear(e, params["mlp.base.0.weight"], params["mlp.base.0.bias"]) * m)
    h = torch.relu(torch.nn.functional.linear(h, params["mlp.base.3.weight"], params["mlp.base.3.bias"]))
    h = torch.relu(torch.nn.functional.linear(h, params["mlp.base.5.weight"], params["mlp.base.5.bias"]))
    sky_ref = torch.nn.functional.linear(h, params["mlp.sh_sky_outlayer.weight"], params["mlp.sh_sky_outlayer.bias"])
    assert torch.allclose(sky.reshape(3, 12), sky_ref, atol=1e-6)
    assert rnd["noise"].shape == (3, 25, 3) and abs(float(rnd["noise"].std()) - 0.025) < 0.01
    assert rnd["dirs"].shape == (3, 10, 3) and float(rnd["dirs"].abs().max()) <= 1.0


@pytest.mark.parametrize("case", [0, 1])
def test_envl_sh_loss(gold, case):
    from gsr import train
    sh = torch.tensor(gold[f"envl{case}/sh"]).requires_grad_(True)
    loss = train.envl_sh_loss(sh, 4, dirs=torch.tensor(gold[f"envl{case}/dirs_unnorm"]))
    want = float(gold[f"envl{case}/loss"])
    got = float(loss.detach())
    assert abs(got - want) <= 1e-5 * max(abs(want), 1e-6), (got, want)
    (d,) = torch.autograd.grad(loss, [sh])
    assert rel_l2(d.numpy(), gold[f"envl{case}/d_sh"]) < 1e-5


def test_envl_sh_loss_zero_when_all_positive():
    from gsr import train
    sh = torch.zeros(1, 25, 3)
    sh[0, 0] = 5.0
    assert float(train.envl_sh_loss(sh, 4, dirs=torch.rand(10, 3) * 2 - 1)) == 0.0


def test_min_scale_and_sky_depth_losses(gold):
    from gsr import train
    scaling = torch.tensor(gold["reg/scaling"]).requires_grad_(True)
    xyz = torch.tensor(gold["reg/xyz"]).requires_grad_(True)
    is_sky = torch.tensor(gold["reg/is_sky"])
    radii = torch.tensor(gold["reg/radii"])
    gs = types.SimpleNamespace(get_scaling=scaling, get_is_sky=is_sky, get_xyz=xyz)
    cam = types.SimpleNamespace(world_view_transform=torch.tensor(gold["reg/viewmatrix"]))
    ms = train.min_scale_loss(radii, gs)
    assert abs(float(ms.detach()) - float(gold["reg/min_scale_loss"])) <= 1e-6 * float(gold["reg/min_scale_loss"])
    (ds,) = torch.autograd.grad(ms, [scaling])
    assert rel_l2(ds.numpy(), gold["reg/d_scaling"]) < 1e-6
    dl = train.depth_loss_gaussians(gs, cam, radii > 0)
    assert abs(float(dl.detach()) - float(gold["reg/depth_loss"])) <= 1e-5 * float(gold["reg/depth_loss"])
    (dx,) = torch.autograd.grad(dl, [xyz])
    assert rel_l2(dx.numpy(), gold["reg/d_xyz"]) < 1e-5


@pytest.mark.parametrize("depth_on", [True, False])
def test_view_regularisers_batched_equal_single_view(depth_on):
    """view_regularisers (all views at once, as train_step runs them) equals the single-view
    reference functions summed as train.py:99-118 adds them: envl_sh_loss unweighted
    (lambda_envlight is a switch), lambda_scale x min_scale_loss, lambda_sky_gauss x
    depth_loss_gaussians only past reg_sky_gauss_depth_from_iter."""
    from gsr import train
    g = torch.Generator().manual_seed(3)
    P, V = 500, 3
    is_sky = torch.rand(P, 1, generator=g) < 0.2
    scaling = (torch.rand(P, 3, generator=g) * 0.1 + 0.01).requires_grad_(True)
    xyz = (torch.randn(P, 3, generator=g) * 2 + torch.tensor([0.0, 0.0, 6.0])).requires_grad_(True)
    pc = types.SimpleNamespace(get_scaling=scaling, get_is_sky=is_sky, get_xyz=xyz)
    radii = torch.randint(0, 3, (V, P), generator=g, dtype=torch.int32)
    vms = torch.eye(4).repeat(V, 1, 1)
    vms[:, 3, :3] = torch.randn(V, 3, generator=g)
    vms[:, :3, :3] = torch.linalg.qr(torch.randn(V, 3, 3, generator=g))[0]
    env = (torch.randn(V, 25, 3, generator=g) * 0.8).requires_grad_(True)
    dirs = torch.rand(V, 10, 3, generator=g) * 2 - 1
    got = train.view_regularisers(pc, radii, vms, env, dirs, depth_on=depth_on)
    assert train.LAMBDA_ENVLIGHT > 0 and train.LAMBDA_SCALE > 0 and train.LAMBDA_SKY_GAUSS > 0
    want = torch.stack([
        train.envl_sh_loss(env[v:v + 1], 4, dirs=dirs[v])
        + train.LAMBDA_SCALE * train.min_scale_loss(radii[v], pc)
        + (train.LAMBDA_SKY_GAUSS * train.depth_loss_gaussians(
            pc, types.SimpleNamespace(world_view_transform=vms[v]), radii[v] > 0) if depth_on else 0.0)
        for v in range(V)])
    assert torch.allclose(got, want, rtol=1e-5, atol=1e-7)
    ins = [scaling, xyz, env] if depth_on else [scaling, env]  # xyz enters only the depth term
    ga = torch.autograd.grad(got.sum(), ins)
    gb = torch.autograd.grad(want.sum(), ins)
    for a, b in zip(ga, gb):
        assert rel_l2(a.numpy(), b.numpy()) < 1e-5


def test_lr_schedule_matches_reference():
    """gsr.train.apply_lr_schedule against the rates the reference's optimizer holds at each
    iteration's step (tests/golden/train_lr.npz from tools/gen_golden_train.py lr: training_setup's
    groups, get_expon_lr_func, GaussianModel / Relightable3DGW.update_learning_rate driven as
    train.py:156-159 drives them), spatial_lr_scale 2.5, with the default MLP rate and with one
    that makes the iteration-20000 reset visible."""
    import numpy as np
    from gsr import train
    d = np.load(os.path.join(os.path.dirname(GOLD), "train_lr.npz"), allow_pickle=False)
    g = torch.Generator().manual_seed(0)
    P_fg, P_sky = 30, 5
    P = P_fg + P_sky
    is_sky = torch.zeros(P, dtype=torch.bool)
    is_sky[P_fg:] = True
    xyz = torch.randn(P, 3, generator=g)
    scale = float(d["lr/spatial_lr_scale"])
    for tag, mlp_lr in (("default", 0.0002), ("mlp1e-3", 0.001)):
        scene = train.RelitScene(xyz, torch.randn(P, 3, generator=g), torch.randn(P, 4, generator=g),
                                 torch.randn(P, 1, generator=g), torch.randn(P_fg, 3, generator=g),
                                 torch.randn(P_fg, 1, generator=g), torch.randn(P_fg, 1, generator=g), is_sky, 2, "cpu",
                                 spatial_lr_scale=scale)
        fp = scene.fp
        for n in fp.names:
            if n == "embeddings" or n.startswith("mlp."):
                fp.set_lr(n, mlp_lr)
        for k, it in enumerate(d["lr/iters"].tolist()):
            train.apply_lr_schedule(scene, it)
            for n, lr in zip(fp.names, fp.lrs):
                ref_name = "mlp" if n.startswith("mlp.") else n
                want = float(d[f"lr/{tag}/{ref_name}"][k])
                assert lr == pytest.approx(want, rel=1e-12), (tag, it, n, lr, want)
