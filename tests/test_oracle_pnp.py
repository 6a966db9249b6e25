"""CPU checks of the SolvePnPWithCV restatement (oracle/pnp.c; g2o_optimization.cc:402-461).
OpenCV is not vendored in the reference (absent here): parity at the OpenCV boundary is
UNPINNED.  Checked instead: the cv::RNG subset sampler against an independent Python
restatement, noise-free known answers, injected-outlier labels, the adaptive iteration
count, and the < 8 correspondence guard."""
import math

import numpy as np
import pytest

import oracle
from rspl_slam_amd import synthetic as SY


def _py_subsets(count, iters):
    s = (1 << 64) - 1
    out = []
    for _ in range(iters):
        sub = []
        while len(sub) < 5:
            s = ((s & 0xFFFFFFFF) * 4164903690 + (s >> 32)) & ((1 << 64) - 1)
            v = (s & 0xFFFFFFFF) % count
            if v not in sub:
                sub.append(v)
        out.append(sub)
    return np.array(out, np.int32)


@pytest.mark.parametrize("count", [8, 57, 300, 2048])
def test_rng_subsets(count):
    np.testing.assert_array_equal(oracle.pnp_subsets(count, 100), _py_subsets(count, 100))


def test_noise_free_known_answer():
    K, X, kp, gt = SY.pnp_problem(n_points=200, pixel_sigma=0.0, outlier_frac=0.0, seed=1)
    n, R, t, inl, used = oracle.pnp(K, X, kp)
    assert n == 200 and inl.all()
    assert np.abs(R - gt["Rwc"]).max() < 1e-6 and np.abs(t - gt["twc"]).max() < 1e-5  # float-rounded inputs
    # all inliers: RANSACUpdateNumIters(0.99, 0, 5, 100) = 0 -> one hypothesis evaluated
    assert used == 1


@pytest.mark.parametrize("seed,outl", [(0, 0.2), (2, 0.4), (3, 0.3)])
def test_outliers_found(seed, outl):
    K, X, kp, gt = SY.pnp_problem(n_points=300, outlier_frac=outl, seed=seed)
    n, R, t, inl, used = oracle.pnp(K, X, kp)
    # gross mismatches (uniform over the image) are far outside 20 px except by chance
    proj_far = np.ones(len(kp), bool)
    Xc = (X - gt["twc"]) @ gt["Rwc"]
    uv = np.stack([K[0] * Xc[:, 0] / Xc[:, 2] + K[2], K[1] * Xc[:, 1] / Xc[:, 2] + K[3]], 1)
    proj_far = np.linalg.norm(kp - uv, axis=1) > 20.0
    np.testing.assert_array_equal(inl == 0, proj_far)
    assert n == int((~proj_far).sum())
    assert np.abs(t - gt["twc"]).max() < 0.02
    p_out = outl
    expect = 100 if math.log(0.01) / math.log(1 - (1 - p_out) ** 5) > 100 else None
    assert used <= 100 and (expect is None or used >= 1)


def test_too_few_points():
    K, X, kp, gt = SY.pnp_problem(n_points=7, outlier_frac=0.0, seed=4)
    n, R, t, inl, used = oracle.pnp(K, X, kp)
    assert n == 0 and used == 0 and not inl.any()


@pytest.mark.parametrize("seed,n,outl", [(0, 300, 0.2), (2, 300, 0.4), (7, 400, 0.25)])
def test_independent_eigen_solver_same_outcome(seed, n, outl):
    """The GPU-mirror eigen order and the independent cyclic Jacobi reach the same RANSAC outcome."""
    K, X, kp, gt = SY.pnp_problem(n_points=n, outlier_frac=outl, seed=seed)
    a, b = oracle.pnp(K, X, kp), oracle.pnp(K, X, kp, independent=True)
    assert a[0] == b[0] and (a[3] == b[3]).all()
    assert np.abs(a[1] - b[1]).max() < 1e-7 and np.abs(a[2] - b[2]).max() < 1e-6
