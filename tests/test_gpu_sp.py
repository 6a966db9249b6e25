"""GPU parity: SuperPoint through the C ABI vs the reference outputs (golden) and the oracle."""
import numpy as np
import pytest

import oracle
import post
from helpers import compare_features

pytestmark = pytest.mark.gpu


def _sp(pkg, w, k, H, W, B=1, thr=0.004, border=4):
    sp = pkg.SuperPoint(pkg.SuperPointConfig(max_keypoints=k, keypoint_threshold=thr, remove_borders=border,
                                             weights=w, max_height=H, max_width=W, max_batch=B))
    assert sp.build(), sp.error
    return sp


@pytest.fixture(scope="module")
def pkg():
    import rspl_loader
    return rspl_loader.load()


def test_sp_small_maps_and_features(pkg, golden, weight_blobs):
    g = golden("sp_small")
    sp = _sp(pkg, weight_blobs[0], 32, 64, 96)
    ok, F = sp.infer(g["image"])
    assert ok, sp.error
    s, d = sp.debug_maps(0, 64, 96)
    np.testing.assert_allclose(d, g["desc"], rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(s, g["scores"], rtol=1e-3, atol=1e-5)
    compare_features(F, g["features"])


def test_sp_euroc_vs_reference(pkg, golden, weight_blobs):
    g = golden("sp_euroc")
    sp = _sp(pkg, weight_blobs[0], 400, 480, 752)
    ok, F = sp.infer(g["image"])
    assert ok, sp.error
    s, d = sp.debug_maps(0, 480, 752)
    nz = np.nonzero(s.reshape(-1))[0]
    np.testing.assert_array_equal(nz, g["nms_idx"])
    np.testing.assert_allclose(s.reshape(-1)[nz], g["nms_val"], rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(d.reshape(-1)[g["desc_sample_idx"]], g["desc_sample_val"], rtol=1e-3, atol=1e-5)
    G = np.concatenate([g["feat_head"], g["feat_desc"].astype(np.float64)])
    compare_features(F, G)


def test_sp_keep_all_and_empty(pkg, weight_blobs):
    from rspl_slam_amd import synthetic as SY
    img = SY.textured_image(96, 128, seed=11, n_blobs=10)
    s, d = oracle.sp_forward(weight_blobs[0], post.image_to_input(img))
    # k = -1: no sort, keypoints in row-major scan order (src/super_point.cpp:193)
    sp = _sp(pkg, weight_blobs[0], -1, 96, 128)
    ok, F = sp.infer(img)
    assert ok, sp.error
    G = post.sp_postprocess(s, d, 0.004, 4, -1)
    compare_features(F, G, order_atol=0.0)   # order is exact (flat index)
    # threshold above every score: zero keypoints
    sp = _sp(pkg, weight_blobs[0], 400, 96, 128, thr=0.99)
    ok, F = sp.infer(img)
    assert ok and F.shape == (259, 0)
    # k larger than the candidate count: all candidates, scan order
    sp = _sp(pkg, weight_blobs[0], 5000, 96, 128)
    ok, F = sp.infer(img)
    compare_features(F, post.sp_postprocess(s, d, 0.004, 4, 5000), order_atol=0.0)


def test_sp_large_border_and_flat_image(pkg, weight_blobs):
    img = np.full((64, 64), 128, np.uint8)     # flat image: plateau scores, NMS ties
    s, d = oracle.sp_forward(weight_blobs[0], post.image_to_input(img))
    sp = _sp(pkg, weight_blobs[0], 50, 64, 64, border=12)
    ok, F = sp.infer(img)
    assert ok, sp.error
    compare_features(F, post.sp_postprocess(s, d, 0.004, 12, 50))


def test_sp_rejects_bad_shapes(pkg, weight_blobs):
    sp = _sp(pkg, weight_blobs[0], 400, 64, 64)
    ok, _ = sp.infer(np.zeros((60, 64), np.uint8))
    assert not ok and "multiples of 8" in sp.error
    ok, _ = sp.infer(np.zeros((72, 64), np.uint8))
    assert not ok


def test_sp_batched_device_path(pkg, weight_blobs):
    from rspl_slam_amd import capi
    from rspl_slam_amd import synthetic as SY
    H, W, k = 480, 752, 400
    left, right = SY.stereo_pair(H, W, seed=3)
    sp = _sp(pkg, weight_blobs[0], k, H, W, B=2)
    st = capi.Stream()
    imgs = capi.DeviceBuffer(2 * H * W).upload(np.stack([left, right]))
    feats = capi.DeviceBuffer(2 * k * 259 * 8)
    counts = capi.DeviceBuffer(2 * 4)
    sp.infer_device(imgs.ptr, 2, H, W, W, H * W, feats.ptr, k, counts.ptr, st.handle)
    st.synchronize()
    F = feats.download((2, k, 259), np.float64)
    cnt = counts.download((2,), np.int32)
    for b, img in enumerate((left, right)):
        s, d = oracle.sp_forward(weight_blobs[0], post.image_to_input(img))
        G = post.sp_postprocess(s, d, 0.004, 4, k)
        compare_features(F[b, :cnt[b]].T, G)


def test_sp_fp16_vs_reference(pkg, golden, weight_blobs):
    """RSPL_PREC_FP16 (the reference's TensorRT kFP16 engine, src/super_point.cpp:98) vs the fp32
    reference outputs, at SURVEY §8c's fp16 acceptance bar: keypoint-set overlap >= 99 % and
    descriptor cosine >= 0.999 on the shared keypoints; scores within 2 %."""
    g = golden("sp_euroc")
    sp = pkg.SuperPoint(pkg.SuperPointConfig(max_keypoints=400, weights=weight_blobs[0], max_height=480,
                                             max_width=752, max_batch=1, precision=pkg.capi.RSPL_PREC_FP16))
    assert sp.build(), sp.error
    ok, F = sp.infer(g["image"])
    assert ok, sp.error
    G = np.concatenate([g["feat_head"], g["feat_desc"].astype(np.float64)])
    kf = {(int(x), int(y)): i for i, (x, y) in enumerate(zip(F[1], F[2]))}
    kg = {(int(x), int(y)): i for i, (x, y) in enumerate(zip(G[1], G[2]))}
    shared = sorted(set(kf) & set(kg))
    overlap = len(shared) / max(1, len(kg))
    fi = np.array([kf[k] for k in shared])
    gi = np.array([kg[k] for k in shared])
    cos = (F[3:, fi] * G[3:, gi]).sum(0) / (np.linalg.norm(F[3:, fi], axis=0) * np.linalg.norm(G[3:, gi], axis=0))
    print(f"fp16 SP: keypoint overlap {overlap:.4f}, min desc cosine {cos.min():.6f}")
    assert overlap >= 0.99
    assert cos.min() >= 0.999
    np.testing.assert_allclose(F[0, fi], G[0, gi], rtol=2e-2, atol=1e-4)


def test_nms_unit_vs_reference(pkg, golden, weight_blobs):
    """The device simple_nms on the reference module's fixture (superpoint.simple_nms, radius 4,
    convert2onnx/superpoint.py:6-33): a random map and two plateau maps with exact ties."""
    g = golden("nms_unit")
    sp = _sp(pkg, weight_blobs[0], 32, 64, 96)
    for k in range(3):
        out = sp.debug_nms(g[f"in{k}"])
        np.testing.assert_array_equal(out, g[f"out{k}"], err_msg=f"map {k}")


def _sp_x3(pkg, w, k, H, W, B=1):
    sp = pkg.SuperPoint(pkg.SuperPointConfig(max_keypoints=k, weights=w, max_height=H, max_width=W, max_batch=B,
                                             precision=pkg.capi.RSPL_PREC_FP16X3))
    assert sp.build(), sp.error
    return sp


def test_sp_fp16x3_vs_reference(pkg, golden, weight_blobs):
    """RSPL_PREC_FP16X3 (split fp16: hi + lo planes, three fp16 MFMA products per step) at the fp32 bar:
    identical keypoint set, scores and descriptors at the fp32 path's tolerances against the reference
    module's outputs (sp_small, sp_euroc)."""
    g = golden("sp_small")
    sp = _sp_x3(pkg, weight_blobs[0], 32, 64, 96)
    ok, F = sp.infer(g["image"])
    assert ok, sp.error
    compare_features(F, g["features"])
    g = golden("sp_euroc")
    sp = _sp_x3(pkg, weight_blobs[0], 400, 480, 752)
    ok, F = sp.infer(g["image"])
    assert ok, sp.error
    G = np.concatenate([g["feat_head"], g["feat_desc"].astype(np.float64)])
    compare_features(F, G)


def test_sp_fp16x3_c1_images_vs_oracle(pkg, weight_blobs):
    """The C1 images (tools/run_c1_plumbing.py: synthetic.stereo_pair seeds 300..) through the split-fp16
    path, batched on the device, against the fp32 oracle: every image's keypoint set identical (the fp16
    path loses 1-5 of 400 keypoints per image near the top-k cut), scores and descriptors at the fp32
    tolerances."""
    from rspl_slam_amd import capi
    H, W, k = 480, 752, 400
    sp = _sp_x3(pkg, weight_blobs[0], k, H, W, B=2)
    imgs = capi.DeviceBuffer(2 * H * W)
    feats, counts = capi.DeviceBuffer(2 * k * 259 * 8), capi.DeviceBuffer(2 * 4)
    st = capi.Stream()
    for t in range(8):
        left, right = pkg.synthetic.stereo_pair(H, W, seed=300 + t)
        imgs.upload(np.stack([left, right]))
        sp.infer_device(imgs.ptr, 2, H, W, W, H * W, feats.ptr, k, counts.ptr, st.handle)
        st.synchronize()
        F = feats.download((2, k, 259), np.float64)
        cnt = counts.download((2,), np.int32)
        for b, img in enumerate((left, right)):
            s, d = oracle.sp_forward(weight_blobs[0], post.image_to_input(img))
            compare_features(F[b, :cnt[b]].T, post.sp_postprocess(s, d, 0.004, 4, k))
