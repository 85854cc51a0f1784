"""CPU checks of the flat-parameter training step plumbing (gsr/train.py): segment layout,
in-place gradient accumulation into the flat buffer (the all-reduce bucket), the losses as
the reference writes them, and the flat gradient's gloo all-reduce (world size 2)."""
import math
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from gsr import train


def test_flat_layout_and_in_place_grads():
    fp = train.FlatParams([("a", (5, 3), 0.1), ("b", (7, 1), 0.2), ("c", (2, 4), 0.3)], "cpu")
    assert fp.offsets == [0, 16, 24] and fp.ends == [16, 24, 32] and fp.n == 32
    fp.load("a", torch.arange(15.0).reshape(5, 3))
    assert torch.equal(fp.flat[:15], torch.arange(15.0))
    for _ in range(2):  # accumulates over two backward passes, into the flat buffer
        loss = (fp.params["a"] ** 2).sum() + 3 * fp.params["b"].sum() + (fp.params["c"] * 2).sum()
        loss.backward()
    fp.check_grads_in_place()
    assert torch.allclose(fp.grad[:15], 4 * torch.arange(15.0))
    assert torch.all(fp.grad[15:16] == 0)  # padding
    assert torch.all(fp.grad[16:23] == 6) and torch.all(fp.grad[24:32] == 4)
    fp.zero_grad()
    assert torch.all(fp.params["a"].grad == 0)


def test_step_requires_gpu():
    fp = train.FlatParams([("a", (4,), 0.1)], "cpu")
    with pytest.raises(RuntimeError):
        fp.step()


def ssim_conv2d(img1, img2, mask=None):
    """utils/loss_utils.py:53-96 restated with torch conv2d (test reference for gsr_ssim)."""
    import torch.nn.functional as F
    c = img1.shape[-3]
    w = train._window(11, c, img1.device)
    a, b = img1[None], img2[None]
    mu1 = F.conv2d(a, w, padding=5, groups=c)
    mu2 = F.conv2d(b, w, padding=5, groups=c)
    mu1_sq, mu2_sq, mu12 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = F.conv2d(a * a, w, padding=5, groups=c) - mu1_sq
    s2 = F.conv2d(b * b, w, padding=5, groups=c) - mu2_sq
    s12 = F.conv2d(a * b, w, padding=5, groups=c) - mu12
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    m = ((2 * mu12 + C1) * (2 * s12 + C2)) / ((mu1_sq + mu2_sq + C1) * (s1 + s2 + C2))
    if mask is None:
        return m.mean()
    return (m * mask[None]).sum() / (mask == 1).sum()


def test_losses_match_reference_formulas():
    g = torch.Generator().manual_seed(0)
    a, b = torch.rand(3, 20, 24, generator=g), torch.rand(3, 20, 24, generator=g)
    m = torch.ones(3, 20, 24)
    m[:, :5] = 0
    # utils/loss_utils.py:27-35
    assert torch.allclose(train.l1_loss(a, b, m), (a * m - b * m).abs().sum() / (m == 1).sum())
    assert torch.allclose(train.l1_loss(a, b), (a - b).abs().mean())
    # the torch restatement the fused GPU SSIM is tested against: 1 for an image with itself
    assert abs(float(ssim_conv2d(a, a, m)) - 1.0) < 1e-5
    assert float(ssim_conv2d(a, b, m)) < 0.5
    with pytest.raises(RuntimeError):  # the product SSIM is the HIP kernel: no CPU path
        train.ssim(a, b, m)
    # the window is the reference's normalised 11-tap Gaussian (sigma 1.5) outer product
    w = train._window(11, 3, "cpu")
    assert w.shape == (3, 1, 11, 11) and abs(float(w[0].sum()) - 1.0) < 1e-6
    g1 = np.array([math.exp(-(x - 5) ** 2 / 4.5) for x in range(11)])
    g1 /= g1.sum()
    assert np.allclose(w[0, 0].numpy(), np.outer(g1, g1), atol=1e-7)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fp = train.FlatParams([("x", (6, 3), 0.1), ("y", (3,), 0.2)], "cpu")
    ((rank + 1) * fp.params["x"].sum() + (rank + 2) * (fp.params["y"] ** 2 + 1).sum()).backward()
    fp.check_grads_in_place()
    dist.all_reduce(fp.grad)  # the training step's one collective, over the flat buffer as is
    # numpy copies travel by value (a torch tensor would travel as a shared-memory file the
    # exiting worker may already have removed)
    q.put((rank, fp.params["x"].grad.numpy().copy(), fp.grad.numpy().copy()))
    dist.destroy_process_group()


def test_flat_grad_all_reduce_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 200
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, gx, gflat in res:
        assert np.all(gx == 3.0)  # 1 + 2
        assert np.array_equal(gflat, res[0][2])
        assert np.all(gflat[20:23] == 0)  # y = 0: d/dy (y^2 + 1) = 0
