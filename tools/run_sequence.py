"""BASELINE C1-style plumbing run: a synthetic 100-keyframe stereo sequence
end to end through the map-side local BA, twice --
  (a) librspl: native Map (csrc/map.cpp) + the GPU LocalmapOptimization, and
  (b) the CPU path: the oracle's restatement of the map (oracle/map_ref.py) + its g2o
      restatement (oracle.ba_local), single-threaded --
with both keyframe trajectories written as TUM files (SaveKeyframeTrajectory, map.cc:1007-1024)
and scored like run_batch.py:48 (evo_ape tum -a): (a) vs (b), each vs ground truth, and the
tracked input vs ground truth.  Prints one JSON line; the TUM files go to --out."""
import argparse
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()
pkg.capi.load()
import map_ref  # noqa: E402  (the CPU path being compared against; test infrastructure)
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
    ap.add_argument("--out", default="gpurun_out/sequence")
    ap.add_argument("--no-cpu", action="store_true", help="GPU path only (stage timing A/B): no oracle run, no ATE")
    a = ap.parse_args()
    from rspl_slam_amd import sequence as SQ, trajectory as TJ
    out = pathlib.Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    seq = pkg.synthetic.map_sequence(n_keyframes=a.keyframes, n_points=a.points, n_lines=a.lines, seed=a.seed,
                                     outlier_frac=0.03)
    ba = pkg.LocalBA(max_poses=32, max_points=a.points + 100, max_lines=a.lines + 10, max_edges=200000)
    if a.analytic_line_jacobian:
        ba.set_line_jacobian(True)
        oracle.ba_set_line_jacobian(True)
    t = time.perf_counter()
    m, reports = SQ.run(seq, ba)
    print(f"gpu path: {len(reports)} keyframes, {time.perf_counter() - t:.2f} s", file=sys.stderr, flush=True)
    gpu_s = time.perf_counter() - t
    m.SaveKeyframeTrajectory(str(out / "keyframe_trajectory_gpu.txt"))
    if a.no_cpu:
        print(json.dumps({"keyframes": len(seq["keyframes"]), "gpu_map_local_ba_ms_per_keyframe":
                          round(gpu_s * 1e3 / (len(seq["keyframes"]) - 1), 3),
                          "gpu_path_ms_per_keyframe": {k: round(float(np.mean([r[k + "_us"] for r in reports])) / 1e3, 3)
                                                       for k in ("insert", "assembly", "ba", "finish")}}))
        return
    t = time.perf_counter()
    mr = map_ref.Map(seq["camera"])
    for k, kf in enumerate(seq["keyframes"]):
        map_ref.insert_keyframe(mr, kf)
        if k:
            map_ref.local_map_optimization(mr, kf["id"], oracle.ba_local)
        if k % 10 == 0:
            print(f"cpu path: keyframe {k}, {time.perf_counter() - t:.1f} s", file=sys.stderr, flush=True)
    cpu_s = time.perf_counter() - t
    (out / "keyframe_trajectory_cpu.txt").write_text("".join(l + "\n" for l in mr.trajectory_lines()))
    tg = TJ.read_tum(str(out / "keyframe_trajectory_gpu.txt"))
    tc = TJ.read_tum(str(out / "keyframe_trajectory_cpu.txt"))
    ts = seq["timestamps"]
    gt = seq["gt_Twc"][:, :3, 3]
    tracked = np.array([kf["Twc"][:3, 3] for kf in seq["keyframes"]])
    res = {"keyframes": len(ts), "points": a.points, "lines": a.lines,
           "analytic_line_jacobian": bool(a.analytic_line_jacobian),
           "ate_gpu_vs_cpu_m": TJ.ape(tc[0], tc[1], tg[0], tg[1])["rmse"],
           "ate_gpu_vs_ground_truth_m": TJ.ape(ts, gt, tg[0], tg[1])["rmse"],
           "ate_cpu_vs_ground_truth_m": TJ.ape(ts, gt, tc[0], tc[1])["rmse"],
           "ate_tracked_input_vs_ground_truth_m": TJ.ape(ts, gt, ts, tracked)["rmse"],
           "tum_files_identical": (out / "keyframe_trajectory_gpu.txt").read_text() ==
           (out / "keyframe_trajectory_cpu.txt").read_text(),
           "point_outliers_removed": int(sum(r["n_point_outliers"] for r in reports)),
           "line_outliers_removed": int(sum(r["n_line_outliers"] for r in reports)),
           "gpu_map_local_ba_ms_per_keyframe": round(gpu_s * 1e3 / (len(ts) - 1), 3),
           "cpu_oracle_ms_per_keyframe_1core": round(cpu_s * 1e3 / (len(ts) - 1), 1),
           # per keyframe: the Python-side insertion, then rspl_map_local_optimization's own stages
           "gpu_path_ms_per_keyframe": {k: round(float(np.mean([r[k + "_us"] for r in reports])) / 1e3, 3)
                                        for k in ("insert", "assembly", "ba", "finish")},
           "window_mean": {k: round(float(np.mean([r[k] for r in reports])), 1)
                           for k in ("n_poses", "n_points", "n_lines", "n_mono", "n_stereo")}}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
