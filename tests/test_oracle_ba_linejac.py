"""Line-edge Jacobians of the BA restatement (oracle/ba.c): g2o's central difference (delta 1e-9, what
EdgeSE3ProjectLine / EdgeStereoSE3ProjectLine get because they do not override linearizeOplus --
include/g2o_optimization/edge_project_line.h:16-31) and its analytic delta -> 0 limit.

The central difference of a line error cancels ~9 digits (terms of ~1e5 px in l2 = Kv . wc against a
2e-9 step), so its Jacobian carries ~1e-7 relative rounding noise that is a pseudo-random function of the
state.  Two runs of the SAME algorithm whose states differ by one ulp -- e.g. the same problem with its
edges handed over in another order -- therefore drift apart on line problems (chi2 ~1e-9, weakly observed
points ~1e-7, Pluecker coordinates ~1e-3), while the analytic limit keeps them within ~1e-11.  These tests
pin (1) the analytic Jacobian to g2o's numeric one, (2) that spread of the reference algorithm itself, which
is the floor any GPU-vs-oracle comparison of line problems in the numeric mode can reach."""
import numpy as np
import pytest

import oracle
from rspl_slam_amd import ba_types as BT
from rspl_slam_amd import synthetic as SY

KINDS = ("mono", "stereo", "mono_line", "stereo_line")


def test_analytic_line_jacobian_matches_central_difference():
    rng = np.random.default_rng(0)
    cam = np.array([435.2047, 435.2047, 367.4517, 252.2009, 47.906])
    worst = 0.0
    for _ in range(200):
        q = rng.normal(size=4)
        q *= np.sign(q[0]) / np.linalg.norm(q)
        t = rng.normal(size=3) * 0.5
        p, d = rng.normal(size=3) + np.array([0, 0, 5.0]), rng.normal(size=3)
        d /= np.linalg.norm(d)
        L = np.concatenate([np.cross(p, d) * rng.uniform(0.5, 2), d * rng.uniform(0.5, 2)])  # unnormalised
        obs = rng.uniform(0, 700, size=8)
        for stereo in (False, True):
            Ja = oracle.line_jacobian(cam, q, t, L, obs, stereo, analytic=True)
            Jn = oracle.line_jacobian(cam, q, t, L, obs, stereo, analytic=False)
            for a, n in zip(Ja, Jn):
                worst = max(worst, float(np.abs(a - n).max() / np.abs(n).max()))
    assert worst < 2e-6, worst  # the central difference's own rounding noise (~1e-7) and nothing else


def _permuted(prob, seed):
    rng = np.random.default_rng(seed)
    perms, kw = {}, {}
    for k in KINDS:
        d = getattr(prob, k)
        perms[k] = rng.permutation(prob.n_edges(k))
        kw[k] = {f: d[f][perms[k]] for f in ("pose", "lm", "cam", "obs")}
    q = BT.DenseProblem(cameras=prob.cameras, pose_q=prob.pose_q, pose_p=prob.pose_p, pose_fixed=prob.pose_fixed,
                        points=prob.points, lines=prob.lines, cfg=prob.cfg, iterations_first=prob.iterations_first,
                        iterations_second=prob.iterations_second, **kw)
    res = oracle.ba_local(q)
    for k in KINDS:
        tmp = res.inlier[k].copy()
        res.inlier[k][perms[k]] = tmp
    return res


@pytest.mark.parametrize("analytic", [False, True])
def test_reference_algorithm_order_spread(analytic):
    """The oracle against itself with the edges permuted (same problem, another summation order)."""
    oracle.ba_set_line_jacobian(analytic)
    try:
        worst = dict(chi2=0.0, pose=0.0, pts=0.0, lines=0.0)
        for c in (dict(n_poses=8, n_points=600, n_lines=20, seed=1, outlier_frac=0.0, init_noise=1.0),
                  dict(n_poses=8, n_points=600, n_lines=30, seed=2, outlier_frac=0.05, init_noise=1.0),
                  dict(n_poses=4, n_points=500, n_lines=10, seed=64, outlier_frac=0.05)):
            p, _ = SY.ba_problem(pixel_sigma=0.8, **c)
            a, b = oracle.ba_local(p), _permuted(p, 3)
            assert (a.iters_first, a.iters_second) == (b.iters_first, b.iters_second)
            for k in KINDS:
                np.testing.assert_array_equal(a.inlier[k], b.inlier[k])
            worst["chi2"] = max(worst["chi2"], abs(a.chi2_second - b.chi2_second) / b.chi2_second,
                                abs(a.chi2_first - b.chi2_first) / b.chi2_first)
            worst["pose"] = max(worst["pose"], float(np.abs(a.pose_p - b.pose_p).max()))
            worst["pts"] = max(worst["pts"], float(np.abs(a.points - b.points).max()))
            worst["lines"] = max(worst["lines"], float(np.abs(a.lines - b.lines).max()))
        print("order spread", "analytic" if analytic else "numeric", worst)
        if analytic:  # smooth in the inputs: rounding-level agreement
            assert worst["chi2"] < 1e-12 and worst["pose"] < 1e-12 and worst["pts"] < 1e-10 and worst["lines"] < 1e-9
        else:  # the central difference's noise: the reference algorithm's own spread (within the GPU bounds)
            assert worst["chi2"] < 5e-8 and worst["pose"] < 1e-6 and worst["pts"] < 1e-5 and worst["lines"] < 5e-3
    finally:
        oracle.ba_set_line_jacobian(False)
