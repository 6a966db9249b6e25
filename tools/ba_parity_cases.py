"""GPU local BA vs the oracle on every problem of tests/test_gpu_ba.py that compares with lines: the actual
differences (chi2 relative, poses, points -- all and those with >= 3 observations -- lines) per case, one JSON
line each (diagnostic for the parity bounds; RSPL_LIB=... for A/B builds)."""
import json
import os
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()
pkg.capi.load()
import oracle  # noqa: E402

SY = pkg.synthetic
ba = pkg.LocalBA(max_poses=40, max_points=12000, max_lines=400, max_edges=80000)
ANALYTIC = "--analytic" in sys.argv  # line Jacobians: analytic limit on both sides (else g2o's central difference)
ba.set_line_jacobian(ANALYTIC)
oracle.ba_set_line_jacobian(ANALYTIC)
cases = []
for s, l, o in [(1, 20, 0.0), (2, 30, 0.05), (3, 0, 0.05), (4, 10, 0.1)]:
    cases.append(("matches_oracle", dict(n_poses=8, n_points=600, n_lines=l, seed=s, pixel_sigma=0.8, outlier_frac=o,
                                         init_noise=1.0), {}))
for n in (23, 33, 36):
    cases.append(("many_poses", dict(n_poses=n, n_points=1500, n_lines=20, seed=40 + n, pixel_sigma=0.8,
                                     outlier_frac=0.05), {}))
cases.append(("long_lines", dict(n_poses=14, n_points=300, n_lines=30, obs_per_point=12, seed=21, pixel_sigma=0.8,
                                 outlier_frac=0.05), {}))
for solver in ("wave", "blk4"):
    for n in (2, 3, 4, 7, 11, 12):
        cases.append(("wave_solve", dict(n_poses=n, n_points=500, n_lines=10, seed=60 + n, pixel_sigma=0.8,
                                         outlier_frac=0.05), {"RSPL_BA_SOLVE": solver}))
cases.append(("reused_result", dict(n_poses=5, n_points=300, n_lines=8, seed=72, pixel_sigma=0.8, outlier_frac=0.05), {}))
cases.append(("euroc_sized", dict(n_poses=10, n_points=4000, n_lines=100, seed=7, pixel_sigma=0.8, outlier_frac=0.05), {}))


def qdiff(a, b):
    s = np.sign((a * b).sum(1, keepdims=True))
    return float(np.abs(a - s * b).max())


for name, c, env in cases:
    os.environ.pop("RSPL_BA_SOLVE", None)
    os.environ.update(env)
    p, _ = SY.ba_problem(**c)
    r, o = ba.run(p), oracle.ba_local(p)
    nobs = np.bincount(np.concatenate([p.mono["lm"], p.stereo["lm"]]), minlength=len(p.points))
    dpt = np.abs(r.points - o.points).max(1) if r.points.size else np.zeros(0)
    rel = lambda a, b: abs(a - b) / max(abs(b), 1e-300)  # noqa: E731
    print(json.dumps({
        "case": name, "line_jac": "analytic" if ANALYTIC else "numeric", **{k: c[k] for k in ("n_poses", "n_points", "n_lines", "seed")}, **env,
        "iters": [r.iters_first, r.iters_second], "iters_oracle": [o.iters_first, o.iters_second],
        "chi2_rel": [rel(r.chi2_first, o.chi2_first), rel(r.chi2_second, o.chi2_second)],
        "pose": max(float(np.abs(r.pose_p - o.pose_p).max()), qdiff(r.pose_q, o.pose_q)),
        "points": float(dpt.max()) if dpt.size else 0.0,
        "points_ge3obs": float(dpt[nobs >= 3].max()) if (nobs >= 3).any() else 0.0,
        "worst_point_nobs": int(nobs[int(dpt.argmax())]) if dpt.size else 0,
        "lines": float(np.abs(r.lines - o.lines).max()) if r.lines.size else 0.0,
        "inliers_equal": all(np.array_equal(r.inlier[k], o.inlier[k]) for k in r.inlier)}), flush=True)
