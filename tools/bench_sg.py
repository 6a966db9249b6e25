"""SuperGlue-only timing on the GPU (bench.py's C3 shape: 2 pairs, 400 keypoints): wall time per
batched call on one stream and the per-stage device times, for one precision."""
import argparse
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()
capi = pkg.capi
capi.load()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", choices=("fp32", "fp16"), default="fp16")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--kpts", type=int, default=400)
    a = ap.parse_args()
    K, B, W, H = a.kpts, 2, 752, 480
    _, sg_w = pkg.weights.ensure_blobs(str(ROOT / "weights"))
    code = capi.RSPL_PREC_FP16 if a.precision == "fp16" else capi.RSPL_PREC_FP32
    sg = pkg.SuperGlue(pkg.SuperGlueConfig(image_width=W, image_height=H, weights=sg_w, max_keypoints=K, max_batch=B,
                                           precision=code))
    assert sg.build(), sg.error
    rng = np.random.default_rng(0)

    def feats():
        f = np.zeros((B, K, 259))
        f[..., 0] = rng.uniform(0.01, 1, (B, K))
        f[..., 1] = rng.uniform(0, W, (B, K))
        f[..., 2] = rng.uniform(0, H, (B, K))
        d = rng.normal(size=(B, K, 256))
        f[..., 3:] = d / np.linalg.norm(d, axis=-1, keepdims=True)
        return f

    FB = K * 259 * 8
    f0, f1 = capi.DeviceBuffer(B * FB), capi.DeviceBuffer(B * FB)
    f0.upload(feats())
    f1.upload(feats())
    n0, n1 = capi.DeviceBuffer(4 * B), capi.DeviceBuffer(4 * B)
    n0.upload(np.full(B, K, np.int32))
    n1.upload(np.full(B, K, np.int32))
    outs = [capi.DeviceBuffer(B * K * sz) for sz in (4, 4, 8, 8)]
    st = capi.Stream()

    def call():
        sg.infer_device(B, f0.ptr, n0.ptr, f1.ptr, n1.ptr, K, True, outs[0].ptr, outs[1].ptr, outs[2].ptr,
                        outs[3].ptr, st.handle)

    for _ in range(5):
        call()
    capi.synchronize()
    sg.profile(True)
    t = time.perf_counter()
    for _ in range(a.iters):
        call()
    capi.synchronize()
    dt = (time.perf_counter() - t) / a.iters * 1e3
    ms, calls = sg.stage_times()
    stages = {k: round(v / max(1, calls), 4) for k, v in zip(pkg.SuperGlue.STAGES, ms)}
    print(f"SG {a.precision} B={B} K={K}: {dt:.3f} ms/call  stages(ms) {stages}")


if __name__ == "__main__":
    main()
