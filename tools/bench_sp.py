"""Quick SuperPoint timing on the GPU: batched device path, HIP events on the kernels' stream."""
import argparse
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()
capi = pkg.capi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--H", type=int, default=480)
    ap.add_argument("--W", type=int, default=752)
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--k", type=int, default=400)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--precision", choices=["fp32", "fp16", "fp16x3"], default="fp16")
    a = ap.parse_args()
    capi.load()
    sp_w, _ = pkg.weights.ensure_blobs(str(ROOT / "weights"))
    sp = pkg.SuperPoint(pkg.SuperPointConfig(max_keypoints=a.k, weights=sp_w, max_height=a.H, max_width=a.W,
                                             max_batch=a.B,
                                             precision={"fp16": capi.RSPL_PREC_FP16, "fp16x3": capi.RSPL_PREC_FP16X3,
                                                        "fp32": capi.RSPL_PREC_FP32}[a.precision]))
    assert sp.build(), sp.error
    st = capi.Stream()
    imgs = capi.DeviceBuffer(a.B * a.H * a.W).upload(
        np.stack([pkg.synthetic.textured_image(a.H, a.W, seed=b) for b in range(a.B)]))
    feats = capi.DeviceBuffer(a.B * a.k * 259 * 8)
    counts = capi.DeviceBuffer(4 * a.B)

    def run():
        sp.infer_device(imgs.ptr, a.B, a.H, a.W, a.W, a.H * a.W, feats.ptr, a.k, counts.ptr, st.handle)

    for _ in range(3):
        run()
    st.synchronize()
    t = capi.Timer()
    t.start(st)
    for _ in range(a.iters):
        run()
    t.stop(st)
    ms = t.elapsed_ms() / a.iters
    gflop = 61.22 * (a.H * a.W) / (480 * 752) * a.B
    print(f"SP B={a.B} {a.H}x{a.W}: {ms:.3f} ms/batch, {gflop / ms:.1f} TFLOP/s (conv), "
          f"counts={counts.download((a.B,), np.int32).tolist()}")


if __name__ == "__main__":
    main()
