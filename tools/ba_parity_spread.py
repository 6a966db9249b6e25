"""GPU local BA vs the oracle on the test problems: relative chi2 differences and max pose / point /
line differences per problem (diagnostic for A/B builds: RSPL_LIB=...)."""
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

ba = pkg.LocalBA(max_poses=40, max_points=12000, max_lines=400, max_edges=80000)
cases = [dict(n_poses=8, n_points=600, n_lines=l, seed=s, pixel_sigma=0.8, outlier_frac=0.05)
         for s, l in ((1, 20), (2, 30), (3, 0), (4, 10))]
cases += [dict(n_poses=5, n_points=300, n_lines=8, seed=72, pixel_sigma=0.8, outlier_frac=0.05),
          dict(n_poses=6, n_points=400, n_lines=12, seed=71, pixel_sigma=0.8, outlier_frac=0.05),
          dict(n_poses=10, n_points=4000, n_lines=100, seed=100)]
for c in cases:
    p, _ = pkg.synthetic.ba_problem(**c)
    r, o = ba.run(p), oracle.ba_local(p)
    rel = lambda a, b: abs(a - b) / abs(b)
    print(f"{c['n_poses']}p {c['n_points']}q {c['n_lines']}l seed {c['seed']}: iters {r.iters_first}+{r.iters_second} "
          f"vs {o.iters_first}+{o.iters_second}  chi2 rel {rel(r.chi2_first, o.chi2_first):.2e} "
          f"{rel(r.chi2_second, o.chi2_second):.2e}  pose {np.abs(r.pose_p - o.pose_p).max():.2e} "
          f"pts {np.abs(r.points - o.points).max():.2e} "
          f"lines {np.abs(r.lines - o.lines).max() if r.lines.size else 0:.2e}", flush=True)
