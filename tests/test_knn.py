"""simple-knn distCUDA2 (submodules/simple-knn/simple_knn.cu:119-220): the C oracle restates
the reference's Morton/box algorithm; CPU tests pin it against brute-force 3-NN, the GPU test
requires bit-identical output from libgsr.so."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc


def brute(pts):
    p = pts.astype(np.float32)
    d = p[None, :, :] - p[:, None, :]
    # the same float op order as the restatement: fma(z, z, fma(y, y, x * x))
    x2 = (d[..., 0] * d[..., 0]).astype(np.float64)
    s = np.float32(np.float32(x2 + np.float64(d[..., 1]) * d[..., 1]) + np.float64(d[..., 2]) * d[..., 2])
    np.fill_diagonal(s, np.inf)
    s.sort(axis=1)
    return ((s[:, 0] + s[:, 1]) + s[:, 2]) / np.float32(3)


def clouds():
    rng = np.random.default_rng(0)
    yield "uniform", rng.uniform(-3, 5, (3000, 3)).astype(np.float32)
    c = rng.normal(0, 1, (20, 3)) * 10
    yield "clusters", (c[rng.integers(0, 20, 2500)] + rng.normal(0, 0.05, (2500, 3))).astype(np.float32)
    yield "plane", np.c_[rng.uniform(0, 1, (1500, 2)), np.zeros(1500)].astype(np.float32)  # degenerate axis
    g = np.stack(np.meshgrid(np.arange(8), np.arange(8), np.arange(8)), -1).reshape(-1, 3).astype(np.float32)
    yield "grid_ties", g
    yield "duplicates", np.repeat(rng.uniform(0, 1, (400, 3)), 3, axis=0).astype(np.float32)


@pytest.mark.parametrize("name,pts", list(clouds()), ids=[n for n, _ in clouds()])
def test_oracle_knn_is_exact_3nn(name, pts):
    got = orc.knn(pts)
    ref = brute(pts)
    np.testing.assert_allclose(got, ref, rtol=2e-6, atol=0)


def test_oracle_knn_tiny():
    got = orc.knn(np.array([[0, 0, 0], [1, 0, 0], [0, 2, 0]], np.float32))
    # fewer than 3 neighbours: the missing slots stay FLT_MAX, so the mean is ~FLT_MAX / 3,
    # as the reference returns (simple_knn.cu:180)
    np.testing.assert_array_equal(got, np.float32(3.402823466e38) / np.float32(3))
    got = orc.knn(np.array([[0, 0, 0], [1, 0, 0], [0, 2, 0], [0, 0, 3]], np.float32))
    np.testing.assert_allclose(got[0], (1 + 4 + 9) / 3.0, rtol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("name,pts", list(clouds()) + [("big", np.random.default_rng(3).normal(0, 4, (200_000, 3))
                                                           .astype(np.float32))],
                         ids=[n for n, _ in clouds()] + ["big"])
def test_distcuda2_bit_exact(name, pts):
    from simple_knn._C import distCUDA2
    got = distCUDA2(torch.tensor(pts, device="cuda")).cpu().numpy()
    ref = orc.knn(pts)
    np.testing.assert_array_equal(got, ref)
