"""Repeat the device-LM BA on seeded problems and compare every run with the oracle (iteration
counts, chi2) -- a race in the trial chain shows up as run-to-run differences."""
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

ba = pkg.LocalBA(max_poses=16, max_points=6000, max_lines=200, max_edges=40000)
bad = 0
for seed, lines, outl in [(4, 10, 0.1), (1, 0, 0.05), (2, 20, 0.1)]:
    prob, _ = pkg.synthetic.ba_problem(n_poses=8, n_points=600, n_lines=lines, seed=seed, pixel_sigma=0.8,
                                       outlier_frac=outl, init_noise=1.0)
    ref = oracle.ba_local(prob)
    runs = [ba.run(prob) for _ in range(30)]
    its = {(r.iters_first, r.iters_second) for r in runs}
    chi = np.array([r.chi2_second for r in runs])
    ok = its == {(ref.iters_first, ref.iters_second)} and np.allclose(chi, ref.chi2_second, rtol=1e-8)
    bad += not ok
    print(seed, lines, outl, "iters", sorted(its), "ref", (ref.iters_first, ref.iters_second),
          "chi2 spread", float(chi.max() - chi.min()), "ok" if ok else "MISMATCH")
sys.exit(1 if bad else 0)
