"""C4 / C5-sized parity (at full size): SuperPoint at BASELINE.json's C4 shape
640x512 and the reference's own OIVIO shape 1280x720 (configs/oivio.yaml:3-4; both k=600) and synthetic 1080x1920 (k=2048), SuperGlue at N=600 and N=2048, and the C5 local BA (30 poses,
10k points, ~6e4 observations) -- the GPU through the C ABI vs the CPU oracle on the same inputs.
The fp16 paths are held to SURVEY §8c's fp16 bar."""
import numpy as np
import pytest

import oracle
import post
from helpers import compare_features, unexplained_match_disagreements
from rspl_slam_amd import synthetic as SY

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pkg():
    import rspl_loader
    return rspl_loader.load()


def _sp(pkg, w, k, H, W, precision=None):
    cfg = pkg.SuperPointConfig(max_keypoints=k, weights=w, max_height=H, max_width=W, max_batch=1)
    if precision is not None:
        cfg.precision = precision
    sp = pkg.SuperPoint(cfg)
    assert sp.build(), sp.error
    return sp


def _restrict_to_common(F, G, score_tol):
    """Top-k at k = 600 / 2048: fp32 accumulation order may swap keypoints tied at the cut.  Every
    keypoint in one set but not the other must score within score_tol of the k-th score; the
    common keypoints are returned (in each matrix's own order) for the full comparison."""
    key = lambda M: [(int(x), int(y)) for x, y in zip(M[1], M[2])]
    kf, kg = key(F), key(G)
    sf, sg = set(kf), set(kg)
    kth = G[0].min() if G.shape[1] else 0.0
    for M, keys, other in ((F, kf, sg), (G, kg, sf)):
        for i, kk in enumerate(keys):
            if kk not in other:
                assert abs(M[0, i] - kth) < score_tol, f"keypoint {kk} (score {M[0, i]}) differs away from the cut"
    common = sf & sg
    return (F[:, [i for i, kk in enumerate(kf) if kk in common]], G[:, [i for i, kk in enumerate(kg) if kk in common]],
            len(common) / max(1, len(sg)))


@pytest.mark.parametrize("H,W,k,seed", [(512, 640, 600, 8), (720, 1280, 600, 4), (1080, 1920, 2048, 5)])
def test_sp_large_vs_oracle(pkg, weight_blobs, H, W, k, seed):
    img = SY.textured_image(H, W, seed=seed, n_blobs=60)
    s, d = oracle.sp_forward(weight_blobs[0], post.image_to_input(img))
    G = post.sp_postprocess(s, d, 0.004, 4, k)
    assert G.shape[1] == k
    sp = _sp(pkg, weight_blobs[0], k, H, W)
    ok, F = sp.infer(img)
    assert ok, sp.error
    Fc, Gc, frac = _restrict_to_common(F, G, 1e-5)
    assert frac > 0.995
    compare_features(Fc, Gc)


@pytest.mark.parametrize("H,W,k,seed", [(512, 640, 600, 8), (1080, 1920, 2048, 5)])
def test_sp_fp16_large(pkg, weight_blobs, H, W, k, seed):
    """fp16 path (the reference's TensorRT kFP16 engine) at C4 (BASELINE.json's 640x512, k=600) and
    C5: keypoint overlap >= 99 %, descriptor cosine >= 0.999 on the common keypoints."""
    img = SY.textured_image(H, W, seed=seed, n_blobs=60)
    s, d = oracle.sp_forward(weight_blobs[0], post.image_to_input(img))
    G = post.sp_postprocess(s, d, 0.004, 4, k)
    sp = _sp(pkg, weight_blobs[0], k, H, W, precision=pkg.capi.RSPL_PREC_FP16)
    ok, F = sp.infer(img)
    assert ok, sp.error
    key = lambda M: {(int(x), int(y)): i for i, (x, y) in enumerate(zip(M[1], M[2]))}
    kf, kg = key(F), key(G)
    common = sorted(set(kf) & set(kg))
    overlap = len(common) / k
    cos = np.array([F[3:, kf[c]] @ G[3:, kg[c]] for c in common])
    print(f"fp16 SP {W}x{H}: overlap {overlap:.4f}, min cosine {cos.min():.6f}")
    assert overlap >= 0.99 and cos.min() >= 0.999


def _features(N, seed):
    rng = np.random.default_rng(seed)
    F = np.zeros((259, N))
    F[0] = rng.uniform(0, 1, N)
    F[1:3] = rng.uniform(-1, 1, (2, N))      # normalised keypoints (PointMatching::NormalizeKeypoints range)
    d = rng.normal(size=(256, N))
    F[3:] = d / np.linalg.norm(d, axis=0)
    return F


def _pair(N, M, seed, frac=0.6, noise=0.15):
    """Two feature sets sharing frac of their keypoints: noisy copies of image-0 descriptors at
    jittered positions, so the assignment has real matches to agree on."""
    rng = np.random.default_rng(seed)
    F0, F1 = _features(N, seed + 1), _features(M, seed + 2)
    m = int(frac * min(N, M))
    a, b = rng.choice(N, m, replace=False), rng.choice(M, m, replace=False)
    d = F0[3:, a] + noise * rng.normal(size=(256, m)) / 16.0
    F1[3:, b] = d / np.linalg.norm(d, axis=0)
    F1[1:3, b] = F0[1:3, a] + 0.005 * rng.normal(size=(2, m))
    return F0, F1


@pytest.mark.parametrize("N,M", [(600, 570), (2048, 2048)])
def test_sg_large_vs_oracle(pkg, weight_blobs, N, M):
    F0, F1 = _pair(N, M, 20 + N)
    k0, s0, d0 = F0[1:3].T, F0[0], F0[3:]
    k1, s1, d1 = F1[1:3].T, F1[0], F1[3:]
    Z = oracle.sg_forward(weight_blobs[1], k0, s0, d0, k1, s1, d1)
    i0r, i1r, m0r, m1r = post.decode(Z)
    res = {}
    for name, prec in (("fp32", pkg.capi.RSPL_PREC_FP32), ("fp16", pkg.capi.RSPL_PREC_FP16)):
        sg = pkg.SuperGlue(pkg.SuperGlueConfig(weights=weight_blobs[1], max_keypoints=max(N, M), max_batch=1,
                                               precision=prec))
        assert sg.build(), sg.error
        ok, i0, i1, m0, m1 = sg.infer(F0, F1)
        assert ok, sg.error
        res[name] = (i0, i1, m0, m1, sg.debug_scores(0, N, M))
    i0, i1, m0, m1, Zg = res["fp32"]
    dz = np.abs(Zg - Z).max()
    print(f"SG N={N}: fp32 max |dZ| vs oracle {dz:.3g}")
    np.testing.assert_allclose(Zg, Z, atol=1e-4, rtol=1e-5)         # Z atol 1e-4
    # indices identical except where the oracle's own Z shows a near-tie within the Z tolerance
    bad = unexplained_match_disagreements(Z, i0, i1, i0r, i1r, tol=2e-4)
    assert not bad, f"{len(bad)} index disagreements not explained by near-ties: {bad[:10]}"
    both = (i0 >= 0) & (i0r >= 0)
    np.testing.assert_allclose(m0[both], m0r[both], atol=1e-3)
    h0, h1 = res["fp16"][0], res["fp16"][1]
    print(f"SG N={N}: fp32 |dZ| {np.abs(Zg - Z).max():.3g}, fp16 agreement {(h0 == i0r).mean():.4f} / "
          f"{(h1 == i1r).mean():.4f}, matches {int((i0r >= 0).sum())}")
    assert (i0r >= 0).sum() > 0.2 * min(N, M)   # the comparison is not vacuous
    assert (h0 == i0r).mean() >= 0.99 and (h1 == i1r).mean() >= 0.99


def test_ba_c5_vs_oracle():
    """C5 local BA: 30 poses (1 fixed), 10k points each seen by 6 poses, stereo/mono mix, 5 % gross
    outliers -- 6K = 174 <= kCholLdsMax = 192: the packed-LDS Schur/LDL^T path."""
    import rspl_loader
    pkg = rspl_loader.load()
    ba = pkg.LocalBA(max_poses=32, max_points=10000, max_lines=16, max_edges=70000)
    prob, gt = SY.ba_problem(n_poses=30, n_points=10000, n_lines=0, seed=5, pixel_sigma=0.8, outlier_frac=0.05)
    res, ref = ba.run(prob), oracle.ba_local(prob)
    assert res.iters_first == ref.iters_first and res.iters_second == ref.iters_second
    np.testing.assert_allclose(res.chi2_first, ref.chi2_first, rtol=1e-8)
    np.testing.assert_allclose(res.chi2_second, ref.chi2_second, rtol=1e-8)
    assert np.abs(res.pose_p - ref.pose_p).max() < 1e-6
    assert np.abs(res.points - ref.points).max() < 1e-5
    for k in res.inlier:
        np.testing.assert_array_equal(res.inlier[k], ref.inlier[k], err_msg=k)
