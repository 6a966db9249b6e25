"""Local-BA timing on the GPU (C3-sized synthetic problems): wall time per LocalmapOptimization call."""
import argparse
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()
pkg.capi.load()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--poses", type=int, default=10)
    ap.add_argument("--points", type=int, default=4000)
    ap.add_argument("--lines", type=int, default=100)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    ba = pkg.LocalBA(max_poses=max(16, a.poses), max_points=a.points + 100, max_lines=a.lines + 10, max_edges=80000)
    probs = [pkg.synthetic.ba_problem(n_poses=a.poses, n_points=a.points, n_lines=a.lines, seed=s)[0] for s in range(3)]
    for p in probs:
        ba.run(p)
    ts = []
    for i in range(a.iters):
        t = time.perf_counter()
        r = ba.run(probs[i % 3])
        ts.append(time.perf_counter() - t)
    dt = float(np.mean(ts)) * 1e3
    e = sum(probs[0].n_edges(k) for k in ("mono", "stereo", "mono_line", "stereo_line"))
    print(f"BA {a.poses} poses {probs[0].points.shape[0]} pts {probs[0].lines.shape[0]} lines {e} edges: "
          f"{dt:.2f} ms/call (median {np.median(ts) * 1e3:.3f} min {np.min(ts) * 1e3:.3f}), "
          f"iters {r.iters_first}+{r.iters_second}")


if __name__ == "__main__":
    main()
