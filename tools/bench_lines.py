"""Line front end timing: the detector (cv::resize + FLD restated: GPU resize /
Sobel / Canny classes + host chaining, rspl_lines_detect) on a 752x480 RCF-like edge map, one
stereo frame's line association -- both images' AssignPointsToLines (one launch) + the stereo
filter + MatchLines (rspl_lines_stereo, host arrays in / out, the reference's per-frame contract)
-- on the GPU, the LineDetector merge passes (host C++), and the oracle restatements of the same
work on one CPU core for comparison."""
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
import fld_ref as FR  # noqa: E402
import lines_ref as LR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=80)
    ap.add_argument("--points", type=int, default=400)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    img, _ = pkg.synthetic.edge_map(seed=11)
    det = pkg.lines.LineDetector()
    for _ in range(5):
        segs = det.detect(img)
    t = time.perf_counter()
    for _ in range(a.iters // 4):
        segs = det.detect(img)
    detect_ms = (time.perf_counter() - t) / (a.iters // 4) * 1e3
    t = time.perf_counter()
    FR.line_detect(img)
    detect_cpu_ms = (time.perf_counter() - t) * 1e3
    sc = pkg.synthetic.line_scene(n_lines=a.lines, n_points=a.points, seed=11)
    lm = pkg.lines.LineMatcher(max_lines=512, max_points=2048)
    lim = (2.0, 60.0, 2.0)
    t = time.perf_counter()
    for _ in range(a.iters):
        L0 = pkg.lines.LineExtractor(sc["seg_left"])
        L1 = pkg.lines.LineExtractor(sc["seg_right"])
    merge_ms = (time.perf_counter() - t) / a.iters * 1e3 / 2
    args = (L0, sc["feat_left"], L1, sc["feat_right"], sc["stereo_matches"], lim)
    for _ in range(10):
        lm.StereoLines(*args)
    t = time.perf_counter()
    for _ in range(a.iters):
        lr, valid, kept = lm.StereoLines(*args)
    gpu_ms = (time.perf_counter() - t) / a.iters * 1e3
    # device-resident form: SuperPoint-layout device features, a device match index per left keypoint
    C = pkg.capi
    m = sc["stereo_matches"]
    cap = max(len(sc["feat_left"]), len(sc["feat_right"]))
    feats = np.zeros((2, cap, 259))
    feats[0, :len(sc["feat_left"])] = sc["feat_left"]
    feats[1, :len(sc["feat_right"])] = sc["feat_right"]
    idx = np.full(cap, -1, np.int32)
    idx[m[:, 0]] = m[:, 1]
    dF = C.DeviceBuffer(feats.nbytes).upload(feats)
    dC = C.DeviceBuffer(8).upload(np.array([len(sc["feat_left"]), len(sc["feat_right"])], np.int32))
    dI = C.DeviceBuffer(idx.nbytes).upload(idx)
    dL0, dL1 = C.DeviceBuffer(L0.nbytes).upload(L0), C.DeviceBuffer(L1.nbytes).upload(L1)
    dO, dV = C.DeviceBuffer(L0.nbytes), C.DeviceBuffer(len(L0))
    st = C.Stream()
    dev = lambda: lm.stereo_lines_device(dL0.ptr, len(L0), dL1.ptr, len(L1), dF.ptr, cap, dC.ptr, dI.ptr, lim,
                                         dO.ptr, dV.ptr, st.handle)
    for _ in range(10):
        dev()
    st.synchronize()
    t = time.perf_counter()
    for _ in range(a.iters):
        dev()
    st.synchronize()
    dev_ms = (time.perf_counter() - t) / a.iters * 1e3
    t = time.perf_counter()
    n_cpu = max(3, a.iters // 50)
    F0, F1, m = sc["feat_left"], sc["feat_right"], sc["stereo_matches"]
    for _ in range(n_cpu):
        km = LR.stereo_filter(F0[:, 1], F1[:, 1], F0[:, 2], F1[:, 2], m, *lim)
        r0 = LR.assign_points_to_lines(L0, F0[:, 1:3])
        r1 = LR.assign_points_to_lines(L1, F1[:, 1:3])
        LR.right_lines(L1, LR.match_lines(r0, r1, km, len(F0), len(F1)), len(L0))
    cpu_ms = (time.perf_counter() - t) / n_cpu * 1e3
    print(json.dumps({"detect_segments": len(segs), "detect_ms_per_image": round(detect_ms, 4),
                      "detect_ms_oracle_python_1core": round(detect_cpu_ms, 2),
                      "lines_left": len(L0), "lines_right": len(L1), "points": a.points,
                      "stereo_matches_kept": kept, "right_lines_valid": int(valid.sum()),
                      "merge_ms_per_image_host": round(merge_ms, 4),
                      "stereo_association_ms_gpu_call": round(gpu_ms, 4),
                      "stereo_association_ms_device_resident": round(dev_ms, 4),
                      "stereo_association_ms_oracle_python_1core": round(cpu_ms, 3)}))


if __name__ == "__main__":
    main()
