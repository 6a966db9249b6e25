"""Is the GPU / oracle trajectory split of a long sequence an implementation defect or a property of the
algorithm?  The CPU oracle path (oracle/map_ref.py + oracle.ba_local, the g2o restatement) is run twice
on the same synthetic sequence: once as is, once with every LocalmapOptimization call's edges handed over
in a fixed random permutation (inlier flags mapped back).  Mathematically the two runs are the same
problem; only the floating-point summation order of chi2 and the normal equations differs -- exactly what
differs between the GPU and the oracle (and between g2o builds with other edge container orders).
Prints the first keyframes whose LM iteration counts, outlier counts or positions differ, and one JSON
summary line (ATE between the two runs, TUM files identical or not).  CPU only; test infrastructure."""
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
import map_ref  # noqa: E402
import oracle  # noqa: E402

KINDS = ("mono", "stereo", "mono_line", "stereo_line")


def permuted_solver(seed):
    rng = np.random.default_rng(seed)

    def solve(prob):
        perms = {}
        kw = {}
        for k in KINDS:
            d = getattr(prob, k)
            n = prob.n_edges(k)
            p = rng.permutation(n)
            perms[k] = p
            kw[k] = {f: d[f][p] for f in ("pose", "lm", "cam", "obs")}
        q = pkg.ba_types.DenseProblem(cameras=prob.cameras, pose_q=prob.pose_q, pose_p=prob.pose_p,
                                      pose_fixed=prob.pose_fixed, points=prob.points, lines=prob.lines,
                                      cfg=prob.cfg, iterations_first=prob.iterations_first,
                                      iterations_second=prob.iterations_second, **kw)
        res = oracle.ba_local(q)
        for k in KINDS:
            tmp = res.inlier[k].copy()
            res.inlier[k][perms[k]] = tmp  # permuted edge i is original edge perm[i]
        return res
    return solve


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keyframes", type=int, default=100)
    ap.add_argument("--points", type=int, default=12000)
    ap.add_argument("--lines", type=int, default=120)
    ap.add_argument("--seed", type=int, default=100)
    ap.add_argument("--perm-seed", type=int, default=7)
    ap.add_argument("--show", type=int, default=4)
    a = ap.parse_args()
    from rspl_slam_amd import trajectory as TJ
    seq = pkg.synthetic.map_sequence(n_keyframes=a.keyframes, n_points=a.points, n_lines=a.lines, seed=a.seed,
                                     outlier_frac=0.03)
    ma, mb = map_ref.Map(seq["camera"]), map_ref.Map(seq["camera"])
    solve_b = permuted_solver(a.perm_seed)
    shown, first = 0, None
    for k, kf in enumerate(seq["keyframes"]):
        map_ref.insert_keyframe(ma, kf)
        map_ref.insert_keyframe(mb, kf)
        if not k:
            continue
        pa, ra, na, nla = map_ref.local_map_optimization(ma, kf["id"], oracle.ba_local)
        pb, rb, nb, nlb = map_ref.local_map_optimization(mb, kf["id"], solve_b)
        ids = [f["id"] for f in seq["keyframes"][:k + 1]]
        dp = max(np.abs(ma.keyframes[i].pose[:3, 3] - mb.keyframes[i].pose[:3, 3]).max() for i in ids)
        sa = (ra.iters_first, ra.iters_second, na, nla)
        sb = (rb.iters_first, rb.iters_second, nb, nlb)
        if sa != sb or dp > 1e-6:
            if first is None:
                first = k
            if shown < a.show:
                print(json.dumps({"keyframe": k, "as_is": sa, "permuted": sb,
                                  "chi2_first": [ra.chi2_first, rb.chi2_first],
                                  "chi2_second": [ra.chi2_second, rb.chi2_second], "max_pos_diff_m": dp}), flush=True)
                shown += 1
        elif k % 10 == 0:
            print(f"keyframe {k}: identical (max pos diff {dp:.2e})", file=sys.stderr, flush=True)
    ta = "".join(l + "\n" for l in ma.trajectory_lines())
    tb = "".join(l + "\n" for l in mb.trajectory_lines())
    out = ROOT / "gpurun_out" / "order_divergence"
    out.mkdir(parents=True, exist_ok=True)
    (out / "as_is.txt").write_text(ta)
    (out / "permuted.txt").write_text(tb)
    A, B = TJ.read_tum(str(out / "as_is.txt")), TJ.read_tum(str(out / "permuted.txt"))
    ts, gt = seq["timestamps"], seq["gt_Twc"][:, :3, 3]
    print(json.dumps({"keyframes": a.keyframes, "points": a.points, "lines": a.lines, "perm_seed": a.perm_seed,
                      "first_divergent_keyframe": first, "tum_files_identical": ta == tb,
                      "ate_permuted_vs_as_is_m": TJ.ape(A[0], A[1], B[0], B[1])["rmse"],
                      "ate_as_is_vs_ground_truth_m": TJ.ape(ts, gt, A[0], A[1])["rmse"],
                      "ate_permuted_vs_ground_truth_m": TJ.ape(ts, gt, B[0], B[1])["rmse"]}))


if __name__ == "__main__":
    main()
