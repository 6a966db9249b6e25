"""Dump FrameOptimization / PnP results of the library RSPL_LIB names (bitwise A/B of two builds):
python tools/experiments/frame_pnp_dump.py OUT.npz"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()
out = {}
probs = [pkg.synthetic.frame_problem(n_points=400, outlier_frac=0.1, seed=s)[0] for s in range(24)]
fba = pkg.FrameBA(max_batch=300, max_edges=300 * 400, max_points=300 * 400)
for tag, batch in (("b1", probs[:1]), ("b24", probs), ("b300", (probs * 13)[:300])):
    res = fba.run(batch)
    out[f"frame_{tag}_pose"] = np.array([np.r_[r.pose_q, r.pose_p] for r in res])
    out[f"frame_{tag}_chi2"] = np.array([r.chi2 for r in res], dtype=np.float64)
    out[f"frame_{tag}_it"] = np.array([r.iterations for r in res])
    out[f"frame_{tag}_inl"] = np.concatenate([np.r_[r.inlier["mono"], r.inlier["stereo"]] for r in res])
frames = [pkg.synthetic.pnp_problem(n_points=400, outlier_frac=0.2, seed=s)[:3] for s in range(16)]
pnp = pkg.PnP(max_batch=16, max_points=16 * 400)
for tag, fr in (("b1", frames[:1]), ("b16", frames)):
    res = pnp.solve(fr)
    out[f"pnp_{tag}_R"] = np.array([r[1] for r in res])
    out[f"pnp_{tag}_t"] = np.array([r[2] for r in res])
    out[f"pnp_{tag}_n"] = np.array([r[0] for r in res])
np.savez(sys.argv[1], **out)
print("dumped", len(out), "arrays")
