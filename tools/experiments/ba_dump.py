"""Dump local-BA results of the library RSPL_LIB names (bitwise A/B of two builds): C3-shaped and C5-shaped
synthetic problems.  python tools/experiments/ba_dump.py OUT.npz"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()
out = {}
for tag, (np_, nq, nl) in (("c3", (10, 4000, 100)), ("c5", (30, 10000, 0))):
    ba = pkg.LocalBA(max_poses=max(16, np_), max_points=nq + 100, max_lines=nl + 10, max_edges=80000)
    for s in range(2):
        r = ba.run(pkg.synthetic.ba_problem(n_poses=np_, n_points=nq, n_lines=nl, seed=s)[0])
        k = f"{tag}_{s}"
        out[k + "_pose"] = np.c_[r.pose_q, r.pose_p]
        out[k + "_points"] = np.array(r.points)
        out[k + "_lines"] = np.array(r.lines)
        out[k + "_chi2"] = np.array([r.chi2_first, r.chi2_second, r.iters_first, r.iters_second])
        out[k + "_inl"] = np.concatenate([np.asarray(r.inlier[q]).ravel() for q in sorted(r.inlier)])
np.savez(sys.argv[1], **out)
print("dumped", len(out), "arrays")
