"""CPU checks of the FrameOptimization restatement (oracle/ba.c orc_frame_opt,
src/g2o_optimization/g2o_optimization.cc:256-398).  g2o is not vendored in the reference, so
parity at the g2o boundary is UNPINNED: the restatement is checked against known answers
(noise-free problems), the injected outlier labels, and an independent optimum -- scipy's
least_squares on the final round's problem (inlier edges, no robust kernel, :363)."""
import numpy as np
import pytest
from scipy.optimize import least_squares
from scipy.spatial.transform import Rotation

import oracle
from rspl_slam_amd import synthetic as SY
from rspl_slam_amd import ba_types as BT


def _Tcw(q_xyzw, p):
    Rwc = Rotation.from_quat(q_xyzw).as_matrix()
    return Rwc.T, -Rwc.T @ p


def test_noise_free_converges_to_ground_truth():
    prob, gt = SY.frame_problem(n_points=200, pixel_sigma=0.0, outlier_frac=0.0, seed=3)
    r = oracle.frame_opt(prob)
    assert r.rounds == 4 and r.n_inliers == 200
    assert np.abs(r.pose_p - gt["pose_p"]).max() < 1e-9
    s = np.sign(np.dot(r.pose_q, gt["pose_q"]))
    assert np.abs(r.pose_q - s * gt["pose_q"]).max() < 1e-9


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_outliers_flagged(seed):
    prob, gt = SY.frame_problem(n_points=300, outlier_frac=0.1, seed=seed)
    r = oracle.frame_opt(prob)
    np.testing.assert_array_equal(r.inlier["mono"] == 0, gt["outlier_mono"])
    np.testing.assert_array_equal(r.inlier["stereo"] == 0, gt["outlier_stereo"])
    assert r.n_inliers == int((~gt["outlier_mono"]).sum() + (~gt["outlier_stereo"]).sum())


@pytest.mark.parametrize("seed", [4, 5])
def test_last_round_is_the_least_squares_optimum(seed):
    prob, gt = SY.frame_problem(n_points=250, outlier_frac=0.08, seed=seed)
    r = oracle.frame_opt(prob)
    cam = prob.cameras[0]
    fx, fy, cx, cy, bf = cam
    mi, si = r.inlier["mono"].astype(bool), r.inlier["stereo"].astype(bool)
    Xm, om = prob.points[prob.mono["lm"][mi]], prob.mono["obs"][mi]
    Xs, os_ = prob.points[prob.stereo["lm"][si]], prob.stereo["obs"][si]

    def resid(x):
        R = Rotation.from_rotvec(x[:3]).as_matrix()
        out = []
        for X, o, st in ((Xm, om, False), (Xs, os_, True)):
            Xc = X @ R.T + x[3:]
            u = fx * Xc[:, 0] / Xc[:, 2] + cx
            v = fy * Xc[:, 1] / Xc[:, 2] + cy
            out += [o[:, 0] - u, o[:, 1] - v]
            if st:
                out.append(o[:, 2] - (u - bf / Xc[:, 2]))
        return np.concatenate(out)

    Rcw, tcw = _Tcw(prob.pose_q, prob.pose_p)
    x0 = np.concatenate([Rotation.from_matrix(Rcw).as_rotvec(), tcw])
    ls = least_squares(resid, x0, method="lm", xtol=1e-15, ftol=1e-15, gtol=1e-15)
    R_ls = Rotation.from_rotvec(ls.x[:3]).as_matrix()
    p_ls = -R_ls.T @ ls.x[3:]
    assert np.abs(r.pose_p - p_ls).max() < 1e-7
    np.testing.assert_allclose(r.chi2[3], (ls.fun ** 2).sum(), rtol=1e-8)


def test_few_edges_single_round():
    prob, gt = SY.frame_problem(n_points=8, outlier_frac=0.0, seed=9)
    r = oracle.frame_opt(prob)
    assert r.rounds == 1  # optimizer.edges().size() < 10 -> break (:383)


def test_no_edges_keeps_pose():
    prob = BT.FrameProblem(cameras=np.array([[435.2, 435.2, 367.4, 252.2, 47.9]]), pose_q=[0, 0, 0, 1],
                           pose_p=[1.0, 2.0, 3.0], points=np.zeros((0, 3)))
    r = oracle.frame_opt(prob)
    assert r.n_inliers == 0 and r.rounds == 1 and r.iterations[0] == 0
    np.testing.assert_allclose(r.pose_p, [1.0, 2.0, 3.0], atol=1e-15)
