"""Host cost of the map side of LocalMapOptimization without a GPU: the synthetic sequence of
tools/run_sequence.py through rspl_map_assemble (window + constraint assembly) and rspl_map_finish
(outlier removal, covisibility update, write-back) with a stand-in BA result -- the assembled state
unchanged and a seeded ~3 % of the constraints flagged as outliers (the sequence's outlier rate).
Prints per-stage means in ms per keyframe (set RSPL_MAP_TIMING=1 for the assembly sub-stages on
stderr)."""
import argparse
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()


def R_to_q(R):
    """rotation matrix -> (x, y, z, w) (Eigen's conversion, as map.cpp R_to_q)"""
    t = np.trace(R)
    q = np.zeros(4)
    if t > 0:
        s = np.sqrt(t + 1.0)
        q[3] = 0.5 * s
        s = 0.5 / s
        q[0] = (R[2, 1] - R[1, 2]) * s
        q[1] = (R[0, 2] - R[2, 0]) * s
        q[2] = (R[1, 0] - R[0, 1]) * s
    else:
        i = int(np.argmax(np.diag(R)))
        j, k = (i + 1) % 3, (i + 2) % 3
        s = np.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0)
        q[i] = 0.5 * s
        s = 0.5 / s
        q[3] = (R[k, j] - R[j, k]) * s
        q[j] = (R[j, i] + R[i, j]) * s
        q[k] = (R[k, i] + R[i, k]) * s
    return q


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keyframes", type=int, default=100)
    ap.add_argument("--points", type=int, default=12000)
    ap.add_argument("--lines", type=int, default=120)
    ap.add_argument("--seed", type=int, default=100)
    a = ap.parse_args()
    from rspl_slam_amd import sequence as SQ
    from rspl_slam_amd.ba_types import DenseResult
    seq = pkg.synthetic.map_sequence(n_keyframes=a.keyframes, n_points=a.points, n_lines=a.lines, seed=a.seed,
                                     outlier_frac=0.03)
    m = pkg.mapping.Map(seq["camera"])
    rng = np.random.default_rng(a.seed)
    t_asm, t_fin, sizes = [], [], []
    for k, kf in enumerate(seq["keyframes"]):
        SQ.insert_keyframe(m, kf)
        if k == 0:
            continue
        t = time.perf_counter()
        rep = m.Assemble(kf["id"])
        t_asm.append(time.perf_counter() - t)
        d = m.LastProblem(rep)
        T = [m.GetPose(int(i)) for i in d["pose_ids"]]
        res = DenseResult(pose_q=np.array([R_to_q(x[:3, :3]) for x in T]).reshape(-1, 4),
                          pose_p=np.array([x[:3, 3] for x in T]).reshape(-1, 3),
                          points=np.array([m.GetMappoint(int(i))[0] for i in d["point_ids"]]).reshape(-1, 3),
                          lines=np.array([m.GetMapline(int(i))[0] for i in d["line_ids"]]).reshape(-1, 6),
                          inlier={kind: (rng.random(len(d[kind]["pose"])) > 0.03).astype(np.uint8)
                                  for kind in ("mono", "stereo", "mono_line", "stereo_line")})
        t = time.perf_counter()
        m.Finish(res)
        t_fin.append(time.perf_counter() - t)
        sizes.append((rep["n_points"], rep["n_mono"] + rep["n_stereo"]))
    print(json.dumps({"keyframes": a.keyframes, "points": a.points,
                      "assembly_ms": round(1e3 * float(np.mean(t_asm)), 3),
                      "finish_ms": round(1e3 * float(np.mean(t_fin)), 3),
                      "window_points_mean": round(float(np.mean([s[0] for s in sizes])), 1),
                      "window_point_edges_mean": round(float(np.mean([s[1] for s in sizes])), 1)}))


if __name__ == "__main__":
    main()
