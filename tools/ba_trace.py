"""Run one seeded BA problem N times with RSPL_BA_LMTRACE set; print the trial traces to stderr."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()
pkg.capi.load()
seed, lines, outl, n = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4])
ba = pkg.LocalBA(max_poses=16, max_points=6000, max_lines=200, max_edges=40000)
prob, _ = pkg.synthetic.ba_problem(n_poses=8, n_points=600, n_lines=lines, seed=seed, pixel_sigma=0.8,
                                   outlier_frac=outl, init_noise=1.0)
for i in range(n):
    r = ba.run(prob)
    print(f"run {i} iters {r.iters_first}+{r.iters_second} chi2 {r.chi2_first:.17g} {r.chi2_second:.17g}", file=sys.stderr)
