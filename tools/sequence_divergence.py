"""Where do the GPU map path and the CPU oracle path of a long synthetic sequence part?  Both run
in lockstep, keyframe by keyframe; per keyframe the BA problem sizes, LM iterations, chi2 and
removed-outlier counts are compared, and the largest keyframe-position difference so far.  Prints
the first keyframes that differ (diagnostic for tools/run_sequence.py)."""
import argparse
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()
pkg.capi.load()
import map_ref  # noqa: E402
import oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keyframes", type=int, default=100)
    ap.add_argument("--points", type=int, default=12000)
    ap.add_argument("--lines", type=int, default=120)
    ap.add_argument("--seed", type=int, default=100)
    ap.add_argument("--analytic-line-jacobian", action="store_true",
                    help="both sides use the analytic limit of g2o's central-difference line Jacobian "
                         "(rspl_ba_set_line_jacobian / oracle.ba_set_line_jacobian)")
    ap.add_argument("--show", type=int, default=6)
    a = ap.parse_args()
    from rspl_slam_amd.sequence import insert_keyframe
    seq = pkg.synthetic.map_sequence(n_keyframes=a.keyframes, n_points=a.points, n_lines=a.lines, seed=a.seed,
                                     outlier_frac=0.03)
    ba = pkg.LocalBA(max_poses=32, max_points=a.points + 100, max_lines=a.lines + 10, max_edges=200000)
    if a.analytic_line_jacobian:
        ba.set_line_jacobian(True)
        oracle.ba_set_line_jacobian(True)
    m = pkg.mapping.Map(seq["camera"])
    mr = map_ref.Map(seq["camera"])
    shown = 0
    for k, kf in enumerate(seq["keyframes"]):
        insert_keyframe(m, kf)
        map_ref.insert_keyframe(mr, kf)
        if not k:
            continue
        rep = m.LocalMapOptimization(kf["id"], ba)
        prob, res, n_out, n_lout = map_ref.local_map_optimization(mr, kf["id"], oracle.ba_local)
        ids = [f["id"] for f in seq["keyframes"][:k + 1]]
        dp = max(np.abs(m.GetPose(i)[:3, 3] - mr.keyframes[i].pose[:3, 3]).max() for i in ids)
        mine = (rep["n_poses"], rep["n_points"], rep["n_mono"] + rep["n_stereo"], rep["iterations_first"],
                rep["iterations_second"], rep["n_point_outliers"], rep["n_line_outliers"])
        ref = (len(prob.pose_q), len(prob.points), prob.n_edges("mono") + prob.n_edges("stereo"), res.iters_first,
               res.iters_second, n_out, n_lout)
        rel = abs(rep["chi2_second"] - res.chi2_second) / max(1e-300, abs(res.chi2_second))
        if mine != ref or dp > 1e-6 or rel > 1e-6:
            print(json.dumps({"keyframe": k, "gpu": mine, "oracle": ref, "chi2_first": [rep["chi2_first"], res.chi2_first],
                              "chi2_second": [rep["chi2_second"], res.chi2_second], "max_pos_diff_m": dp}), flush=True)
            shown += 1
            if shown >= a.show:
                break
        elif k % 10 == 0:
            print(f"keyframe {k}: identical (max pos diff {dp:.2e})", flush=True)


if __name__ == "__main__":
    main()
