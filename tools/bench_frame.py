"""FrameOptimization timing on the GPU: latency of one frame (the reference's per-frame tracking
call, map_builder.cc:583) and throughput of a batch of independent frames in one launch
(C4 shape: many sequences per GPU), beside the oracle's fp64 C restatement on one host core."""
import argparse
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()
pkg.capi.load()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=400)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    probs = [pkg.synthetic.frame_problem(n_points=a.points, outlier_frac=0.1, seed=s)[0] for s in range(a.batch)]
    fba = pkg.FrameBA(max_batch=a.batch, max_edges=a.batch * a.points, max_points=a.batch * a.points)
    out = {"points_per_frame": a.points}
    import ctypes as C
    from rspl_slam_amd import ba_types as BT
    res = [BT.FrameResult.alloc(p) for p in probs]
    P = (BT.RsplFrameProblem * a.batch)(*[p.to_ctypes() for p in probs])   # marshalled once
    R = (BT.RsplFrameResult * a.batch)(*[r.to_ctypes() for r in res])
    lib = pkg.capi.load()
    for b in (1, a.batch):
        pkg.capi.check(lib.rspl_frame_optimize(fba._h, P, b, R), "rspl_frame_optimize")
        t = time.perf_counter()
        for _ in range(a.iters):
            lib.rspl_frame_optimize(fba._h, P, b, R)
        dt = (time.perf_counter() - t) / a.iters
        out[f"batch{b}_ms_per_call"] = round(dt * 1e3, 3)
        out[f"batch{b}_frames_per_s"] = round(b / dt, 1)
    import oracle  # CPU baseline only
    t = time.perf_counter()
    n = 0
    while time.perf_counter() - t < 2.0:
        oracle.frame_opt(probs[n % a.batch])
        n += 1
    out["cpu_oracle_1core_frames_per_s"] = round(n / (time.perf_counter() - t), 1)
    # SolvePnPWithCV (the per-frame initial pose before FrameOptimization, map_builder.cc:515)
    frames = [pkg.synthetic.pnp_problem(n_points=a.points, outlier_frac=0.2, seed=s)[:3] for s in range(128)]
    pnp = pkg.PnP(max_batch=128, max_points=128 * a.points)
    for b in (1, 128):
        pnp.solve(frames[:b])
        t = time.perf_counter()
        for _ in range(a.iters):
            pnp.solve(frames[:b])
        dt = (time.perf_counter() - t) / a.iters
        out[f"pnp_batch{b}_ms_per_call"] = round(dt * 1e3, 3)
        out[f"pnp_batch{b}_frames_per_s"] = round(b / dt, 1)
    t = time.perf_counter()
    n = 0
    while time.perf_counter() - t < 2.0:
        oracle.pnp(*frames[n % 128])
        n += 1
    out["pnp_cpu_oracle_1core_frames_per_s"] = round(n / (time.perf_counter() - t), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
