"""GPU parity: SuperGlue / PointMatching through the C ABI vs the reference outputs (golden) and the oracle."""
import numpy as np
import pytest

import oracle
import post

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pkg():
    import rspl_loader
    return rspl_loader.load()


def _sg(pkg, w, nmax=400, B=1):
    sg = pkg.SuperGlue(pkg.SuperGlueConfig(weights=w, max_keypoints=nmax, max_batch=B))
    assert sg.build(), sg.error
    return sg


@pytest.mark.parametrize("name,atol", [("sg_small", 1e-4), ("sg_400", 1e-4)])   # Z atol 1e-4
def test_sg_vs_reference(pkg, golden, weight_blobs, name, atol):
    g = golden(name)
    F0, F1 = g["F0"].astype(np.float64), g["F1"].astype(np.float64)
    G0, G1 = post.normalize_keypoints(F0, 752, 480), post.normalize_keypoints(F1, 752, 480)
    sg = _sg(pkg, weight_blobs[1], nmax=max(F0.shape[1], F1.shape[1]))
    ok, i0, i1, m0, m1 = sg.infer(G0, G1)
    assert ok, sg.error
    Z = sg.debug_scores(0, F0.shape[1], F1.shape[1])
    print(f"{name}: max |dZ| vs the reference module {np.abs(Z - g['Z']).max():.3g}")
    np.testing.assert_allclose(Z, g["Z"], atol=atol, rtol=1e-5)
    np.testing.assert_array_equal(i0, g["idx0"])
    np.testing.assert_array_equal(i1, g["idx1"])
    np.testing.assert_allclose(m0, g["ms0"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(m1, g["ms1"], rtol=1e-4, atol=1e-6)
    # decode on our own Z must be exactly the restated reference decode
    d = post.decode(Z)
    np.testing.assert_array_equal(i0, d[0])
    np.testing.assert_array_equal(i1, d[1])
    np.testing.assert_allclose(m0, d[2], rtol=2e-7, atol=0)


def test_point_matching_vs_reference(pkg, golden, weight_blobs):
    g = golden("sg_400")
    pm = pkg.PointMatching(pkg.SuperGlueConfig(weights=weight_blobs[1], max_keypoints=400, max_batch=1))
    n, matches = pm.MatchingPoints(g["F0"].astype(np.float64), g["F1"].astype(np.float64))
    assert n == len(g["matches"])
    np.testing.assert_array_equal(np.array([(q, t) for q, t, _ in matches]), g["matches"])
    np.testing.assert_allclose(np.array([d for _, _, d in matches]), g["distances"], atol=1e-5)


def test_sg_ragged_and_empty(pkg, weight_blobs):
    from rspl_slam_amd import synthetic as SY
    sg = _sg(pkg, weight_blobs[1], nmax=96)
    for n0, n1 in [(1, 1), (1, 7), (33, 5), (96, 95), (64, 64)]:
        F0, F1, _ = SY.sg_problem(n0, n1, min(n0, n1) // 2, seed=n0 * 100 + n1)
        G0, G1 = post.normalize_keypoints(F0, 752, 480), post.normalize_keypoints(F1, 752, 480)
        ok, i0, i1, m0, m1 = sg.infer(G0, G1)
        assert ok, sg.error
        Zo = oracle.sg_forward(weight_blobs[1], *post.sg_inputs(G0), *post.sg_inputs(G1))
        Z = sg.debug_scores(0, n0, n1)
        np.testing.assert_allclose(Z, Zo, atol=1e-4, rtol=1e-5, err_msg=f"{n0}x{n1}")
        d = post.decode(Z)
        np.testing.assert_array_equal(i0, d[0])
        np.testing.assert_array_equal(i1, d[1])
    F0, _, _ = SY.sg_problem(8, 8, 4, seed=1)
    ok, i0, i1, m0, m1 = sg.infer(F0, np.zeros((259, 0)))
    assert ok and (i0 == -1).all() and (m0 == 0).all() and i1.size == 0
    ok, *_ = sg.infer(np.zeros((259, 97)), F0)        # above max_keypoints: rejected
    assert not ok


def test_sg_batched_device_path(pkg, weight_blobs):
    from rspl_slam_amd import capi
    from rspl_slam_amd import synthetic as SY
    nmax, B = 400, 2
    probs = [SY.sg_problem(400, 380, 300, seed=10), SY.sg_problem(350, 400, 200, seed=11)]
    sg = _sg(pkg, weight_blobs[1], nmax=nmax, B=B)
    f0 = np.zeros((B, nmax, 259)); f1 = np.zeros((B, nmax, 259))
    n0 = np.zeros(B, np.int32); n1 = np.zeros(B, np.int32)
    for p, (F0, F1, _) in enumerate(probs):
        f0[p, :F0.shape[1]] = F0.T; f1[p, :F1.shape[1]] = F1.T
        n0[p], n1[p] = F0.shape[1], F1.shape[1]
    st = capi.Stream()
    bufs = {k: capi.DeviceBuffer(v.nbytes).upload(v) for k, v in dict(f0=f0, f1=f1, n0=n0, n1=n1).items()}
    out = {k: capi.DeviceBuffer(B * nmax * sz) for k, sz in dict(i0=4, i1=4, m0=8, m1=8).items()}
    sg.infer_device(B, bufs["f0"].ptr, bufs["n0"].ptr, bufs["f1"].ptr, bufs["n1"].ptr, nmax, True,
                    out["i0"].ptr, out["i1"].ptr, out["m0"].ptr, out["m1"].ptr, st.handle)
    st.synchronize()
    I0 = out["i0"].download((B, nmax), np.int32)
    I1 = out["i1"].download((B, nmax), np.int32)
    for p, (F0, F1, _) in enumerate(probs):
        G0, G1 = post.normalize_keypoints(F0, 752, 480), post.normalize_keypoints(F1, 752, 480)
        Zo = oracle.sg_forward(weight_blobs[1], *post.sg_inputs(G0), *post.sg_inputs(G1))
        d = post.decode(Zo)
        np.testing.assert_array_equal(I0[p, :n0[p]], d[0])
        np.testing.assert_array_equal(I1[p, :n1[p]], d[1])


def test_sg_fp16_vs_reference(pkg, golden, weight_blobs):
    """RSPL_PREC_FP16 (the reference's TensorRT kFP16 engine, src/super_glue.cpp:132) vs the fp32
    reference at SURVEY §8c's fp16 bar: match-index agreement >= 99 %."""
    g = golden("sg_400")
    F0, F1 = g["F0"].astype(np.float64), g["F1"].astype(np.float64)
    G0, G1 = post.normalize_keypoints(F0, 752, 480), post.normalize_keypoints(F1, 752, 480)
    sg = pkg.SuperGlue(pkg.SuperGlueConfig(weights=weight_blobs[1], max_keypoints=400, max_batch=1,
                                           precision=pkg.capi.RSPL_PREC_FP16))
    assert sg.build(), sg.error
    ok, i0, i1, m0, m1 = sg.infer(G0, G1)
    assert ok, sg.error
    Z = sg.debug_scores(0, F0.shape[1], F1.shape[1])
    agree0 = (i0 == g["idx0"]).mean()
    agree1 = (i1 == g["idx1"]).mean()
    zerr = np.abs(Z - g["Z"]).max()
    print(f"fp16 SG: idx0 agreement {agree0:.4f}, idx1 {agree1:.4f}, max |dZ| {zerr:.4g}, "
          f"matches {int((i0 >= 0).sum())} vs {int((g['idx0'] >= 0).sum())}")
    assert agree0 >= 0.99 and agree1 >= 0.99
    both = (i0 >= 0) & (g["idx0"] >= 0)
    np.testing.assert_allclose(m0[both], g["ms0"][both], atol=2e-2)


def test_sg_post_stream_pipelined(pkg, weight_blobs):
    """rspl_sg_infer_device2: Sinkhorn + decode on a second stream, 4 calls back to back with the
    count buffers overwritten right after each call (parity double-buffering + count snapshot);
    every call's indices equal the single-stream result of the same inputs."""
    from rspl_slam_amd import capi
    from rspl_slam_amd import synthetic as SY
    nmax, B = 400, 2
    sg = _sg(pkg, weight_blobs[1], nmax=nmax, B=B)
    calls = []
    for c in range(4):
        probs = [SY.sg_problem(400 - 20 * c, 380, 250, seed=30 + c), SY.sg_problem(300 + 10 * c, 400, 200, seed=40 + c)]
        f0 = np.zeros((B, nmax, 259)); f1 = np.zeros((B, nmax, 259))
        n0 = np.zeros(B, np.int32); n1 = np.zeros(B, np.int32)
        for p, (F0, F1, _) in enumerate(probs):
            f0[p, :F0.shape[1]] = F0.T; f1[p, :F1.shape[1]] = F1.T
            n0[p], n1[p] = F0.shape[1], F1.shape[1]
        calls.append((f0, f1, n0, n1))

    def run(post):
        st, pst = capi.Stream(), capi.Stream()
        fb = [capi.DeviceBuffer(calls[0][0].nbytes) for _ in range(2)]
        cb = [capi.DeviceBuffer(8) for _ in range(2)]
        outs = [{k: capi.DeviceBuffer(B * nmax * sz) for k, sz in dict(i0=4, i1=4, m0=8, m1=8).items()}
                for _ in calls]
        for c, (f0, f1, n0, n1) in enumerate(calls):
            st.synchronize()
            fb[0].upload(f0); fb[1].upload(f1); cb[0].upload(n0); cb[1].upload(n1)
            o = outs[c]
            sg.infer_device(B, fb[0].ptr, cb[0].ptr, fb[1].ptr, cb[1].ptr, nmax, True, o["i0"].ptr, o["i1"].ptr,
                            o["m0"].ptr, o["m1"].ptr, st.handle, post_stream=pst.handle if post else None)
            if post:  # overwrite the counts as soon as the main stream has passed the call
                st.synchronize()
                cb[0].upload(np.zeros(B, np.int32)); cb[1].upload(np.zeros(B, np.int32))
        capi.synchronize()
        return [(o["i0"].download((B, nmax), np.int32), o["i1"].download((B, nmax), np.int32)) for o in outs]

    ref, got = run(False), run(True)
    for (a0, a1), (b0, b1) in zip(ref, got):
        np.testing.assert_array_equal(a0, b0)
        np.testing.assert_array_equal(a1, b1)


def test_sinkhorn_unit_vs_reference(pkg, golden, weight_blobs):
    """The device log-Sinkhorn on the reference module's own fixture (superglue.log_optimal_transport,
    convert2onnx/superglue.py:185-205: random 64x56 scores, bin score alpha, 100 iterations)."""
    g = golden("sinkhorn_unit")
    sg = _sg(pkg, weight_blobs[1], nmax=64)
    ok, Z = sg.debug_sinkhorn(g["scores"], float(g["alpha"]), int(g["iters"]))
    assert ok, sg.error
    print(f"sinkhorn_unit: max |dZ| {np.abs(Z - g['Z']).max():.3g}")
    np.testing.assert_allclose(Z, g["Z"], atol=1e-4, rtol=0)
    i0, i1, m0, m1 = sg.debug_decode(Z)
    np.testing.assert_array_equal(i0, g["idx0"])
    np.testing.assert_array_equal(i1, g["idx1"])
    np.testing.assert_allclose(m0, g["ms0"], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("which", ["Z", "Z_ties"])
def test_decode_unit_vs_reference(pkg, golden, weight_blobs, which):
    """The device decode (argmax / col_argmax / finalize) on the reference's decode fixtures, including
    Z_ties (duplicated row / column maxima: first maximum wins, src/super_glue.cpp:258-337)."""
    g = golden("sinkhorn_unit")
    sg = _sg(pkg, weight_blobs[1], nmax=64)
    i0, i1, m0, m1 = sg.debug_decode(g[which])
    p = "" if which == "Z" else "t_"
    np.testing.assert_array_equal(i0, g[p + "idx0"])
    np.testing.assert_array_equal(i1, g[p + "idx1"])
    # std::exp(float) widened to double: the device expf and the fixture's exp agree to 1 float ulp
    np.testing.assert_allclose(m0, g[p + "ms0"], rtol=2.4e-7, atol=0)
    np.testing.assert_allclose(m1, g[p + "ms1"], rtol=2.4e-7, atol=0)


def test_sinkhorn_timeout_reaches_caller(pkg, weight_blobs):
    """A Sinkhorn exchange timeout (injected) is reported on the device path through rspl_sg_status and
    fails rspl_sg_infer; clearing the injection restores correct results on the same handle."""
    from rspl_slam_amd import capi
    from rspl_slam_amd import synthetic as SY
    sg = _sg(pkg, weight_blobs[1], nmax=96, B=2)
    F0, F1, _ = SY.sg_problem(90, 80, 40, seed=3)
    G0, G1 = post.normalize_keypoints(F0, 752, 480), post.normalize_keypoints(F1, 752, 480)
    ok, r0, r1, _, _ = sg.infer(G0, G1)
    assert ok, sg.error
    sg.debug_inject(True, spin_limit=1 << 12)
    ok, *_ = sg.infer(G0, G1)
    assert not ok and "timed out" in sg.error
    # device path: the flag is sticky until rspl_sg_status reads it
    nmax, B = 96, 2
    f0 = np.zeros((B, nmax, 259)); f1 = np.zeros((B, nmax, 259))
    f0[:, :90] = G0.T; f1[:, :80] = G1.T
    st = capi.Stream()
    bufs = {k: capi.DeviceBuffer(v.nbytes).upload(v) for k, v in
            dict(f0=f0, f1=f1, n0=np.array([90, 90], np.int32), n1=np.array([80, 80], np.int32)).items()}
    out = {k: capi.DeviceBuffer(B * nmax * sz) for k, sz in dict(i0=4, i1=4, m0=8, m1=8).items()}
    sg.infer_device(B, bufs["f0"].ptr, bufs["n0"].ptr, bufs["f1"].ptr, bufs["n1"].ptr, nmax, False,
                    out["i0"].ptr, out["i1"].ptr, out["m0"].ptr, out["m1"].ptr, st.handle)
    st.synchronize()
    ok, mask = sg.status()
    assert not ok and mask & 1, (ok, mask)
    assert sg.status() == (True, 0)          # cleared by the read
    sg.debug_inject(False)
    ok, i0, i1, _, _ = sg.infer(G0, G1)
    assert ok, sg.error
    np.testing.assert_array_equal(i0, r0)
    np.testing.assert_array_equal(i1, r1)
    assert sg.status() == (True, 0)


@pytest.mark.parametrize("kernel,G", [("slab", None), ("sc", 4), ("sc", 8), ("sc", 16), ("sc", 32)])
def test_sinkhorn_kernels_vs_reference(pkg, golden, weight_blobs, monkeypatch, kernel, G):
    """Every Sinkhorn kernel (the slab kernel: row + column slabs in LDS, two all-gathers per
    iteration; the scaling-form kernel, the default: whole rows of register-resident
    exp(C + a + b), one all-gather of per-column partial sums per iteration) at every instantiated
    rows-per-wave, on the reference module's fixtures (superglue.log_optimal_transport,
    convert2onnx/superglue.py:185-205): Z at atol 1e-4, identical matches.  RSPL_SG_SINK /
    RSPL_SG_SINK_G are read when the handle is created."""
    monkeypatch.setenv("RSPL_SG_SINK", kernel)
    if G:
        monkeypatch.setenv("RSPL_SG_SINK_G", str(G))
    g = golden("sinkhorn_unit")
    sg = _sg(pkg, weight_blobs[1], nmax=64)
    ok, Z = sg.debug_sinkhorn(g["scores"], float(g["alpha"]), int(g["iters"]))
    assert ok, sg.error
    np.testing.assert_allclose(Z, g["Z"], atol=1e-4, rtol=0)
    for it in (0, 1, 3):  # short runs, incl. no iteration at all (Z = C - norm): the oracle's restatement
        ok, Z = sg.debug_sinkhorn(g["scores"], float(g["alpha"]), it)
        assert ok, sg.error
        np.testing.assert_allclose(Z, oracle.log_optimal_transport(g["scores"], float(g["alpha"]), it),
                                   atol=1e-4, rtol=0)
    g = golden("sg_400")
    F0, F1 = g["F0"].astype(np.float64), g["F1"].astype(np.float64)
    G0, G1 = post.normalize_keypoints(F0, 752, 480), post.normalize_keypoints(F1, 752, 480)
    sg = _sg(pkg, weight_blobs[1], nmax=max(F0.shape[1], F1.shape[1]))
    ok, i0, i1, m0, m1 = sg.infer(G0, G1)
    assert ok, sg.error
    Z = sg.debug_scores(0, F0.shape[1], F1.shape[1])
    print(f"{kernel} G={G}: max |dZ| vs the reference module {np.abs(Z - g['Z']).max():.3g}")
    np.testing.assert_allclose(Z, g["Z"], atol=1e-4, rtol=1e-5)
    np.testing.assert_array_equal(i0, g["idx0"])
    np.testing.assert_array_equal(i1, g["idx1"])


def test_sinkhorn_scaling_absorption(pkg, weight_blobs):
    """The scaling-form kernel on couplings with a large dynamic range (scores ~ N(0, 30)): its
    scalings leave [2^-60, 2^60] and are absorbed into the log potentials (K rebuilt from C);
    Z must still equal the oracle's log-domain Sinkhorn at atol 1e-4 (|Z| reaches hundreds)."""
    rng = np.random.default_rng(3)
    S = (rng.normal(size=(300, 280)) * 30).astype(np.float32)
    sg = _sg(pkg, weight_blobs[1], nmax=300)
    ok, Z = sg.debug_sinkhorn(S, 1.0, 100)
    assert ok, sg.error
    Zr = oracle.log_optimal_transport(S, 1.0, 100)
    np.testing.assert_allclose(Z, Zr, atol=2e-4 * max(1.0, np.abs(Zr).max() / 100), rtol=0)


@pytest.mark.parametrize("G,scale", [(None, 1.0), (16, 1.0), (None, 30.0)])
def test_sinkhorn_sc10_vs_oracle(pkg, weight_blobs, monkeypatch, G, scale):
    """The scaling-form kernel's wide instantiation (448 < nmax + 1 <= 640: ten 64-column sets per
    lane, <= 48 rows per workgroup, the column exchange in two passes above 512 columns) -- C4's
    600 keypoints -- against the oracle's log-domain Sinkhorn (superglue.py:185-205) on a 600 x 570
    score matrix; scale 30 forces scaling absorption.  Z at atol 1e-4 (scaled with |Z| as above)."""
    if G:
        monkeypatch.setenv("RSPL_SG_SINK_G", str(G))
    rng = np.random.default_rng(11)
    S = (rng.normal(size=(600, 570)) * scale).astype(np.float32)
    sg = _sg(pkg, weight_blobs[1], nmax=600)
    ok, Z = sg.debug_sinkhorn(S, 1.0, 100)
    assert ok, sg.error
    Zr = oracle.log_optimal_transport(S, 1.0, 100)
    print(f"sc10 G={G} scale={scale}: max |dZ| {np.abs(Z - Zr).max():.3g}")
    np.testing.assert_allclose(Z, Zr, atol=1e-4 * max(1.0, 2 * np.abs(Zr).max() / 100), rtol=0)


@pytest.mark.parametrize("M,N,scale", [(2048, 1900, 1.0), (2048, 2048, 30.0), (1500, 2048, 1.0)])
def test_sinkhorn_wide_vs_oracle(pkg, weight_blobs, M, N, scale):
    """The wide scaling-form kernel (640 < nmax + 1 <= 2112: C5's 2048 keypoints, 65 workgroups per pair,
    the column exchange in two hops -- reduce-scatter to the column owners, broadcast of V) against the
    oracle's log-domain Sinkhorn (superglue.py:185-205), incl. a run that forces scaling absorption
    (scale 30) and pairs smaller than nmax in either dimension.  Z at atol 1e-4, scaled with max |Z| as
    the 600-column test above but by 3 instead of 2: an error of the potentials u_i / v_j shifts whole
    rows / columns of Z, and it grows with the fp32 rounding of the 2049-term sums (sqrt(2049 / 571) ~ 1.9x
    the 600-column case: measured 5.6e-4 at max |Z| ~270 vs 1.9e-4 there); at scale 1, max |dZ| 4.8e-6."""
    rng = np.random.default_rng(21)
    S = (rng.normal(size=(M, N)) * scale).astype(np.float32)
    sg = _sg(pkg, weight_blobs[1], nmax=2048)
    ok, Z = sg.debug_sinkhorn(S, 1.0, 100)
    assert ok, sg.error
    assert sg.status() == (True, 0)
    Zr = oracle.log_optimal_transport(S, 1.0, 100)
    print(f"wide {M}x{N} scale={scale}: max |dZ| {np.abs(Z - Zr).max():.3g}")
    np.testing.assert_allclose(Z, Zr, atol=1e-4 * max(1.0, 3 * np.abs(Zr).max() / 100), rtol=0)
    for it in (0, 1):  # short runs incl. no iteration (Z = C - norm)
        ok, Z = sg.debug_sinkhorn(S, 1.0, it)
        assert ok, sg.error
        np.testing.assert_allclose(Z, oracle.log_optimal_transport(S, 1.0, it), atol=1e-4, rtol=0)


def _pm(pkg, blob, precision):
    return pkg.PointMatching(pkg.SuperGlueConfig(image_width=752, image_height=480, weights=blob, max_keypoints=400,
                                                 max_batch=1, precision=precision))


def test_sg_c1_stereo_pair_fp32(pkg, golden, sg_c1_blob):
    """The C1 stereo pair's SuperPoint features (reference modules) through PointMatching on the GPU at
    fp32 with the "c1" SuperGlue profile: Z and the assignment probabilities vs the reference module
    (the profile's sharper scores scale fp32 accumulation noise with |Z|, which reaches ~870 here: Z atol
    1.5e-3 + rtol 1e-4, measured 3.4e-3 at rel 8.5e-5; the probabilities exp(Z) at atol 1e-4 + rtol 5e-4,
    since dp = p dZ: measured 1.3e-4 at p ~ 0.6),
    identical decode and a NON-EMPTY thresholded DMatch list identical to the reference's
    (point_matching.cc:12-48, super_glue.cpp:339-367), distances within the probability tolerance."""
    g = golden("sg_c1")
    F0, F1 = g["F0"].astype(np.float64), g["F1"].astype(np.float64)
    pm = _pm(pkg, sg_c1_blob, pkg.capi.RSPL_PREC_FP32)
    n, ml = pm.MatchingPoints(F0, F1)
    Z = pm.superglue.debug_scores(0, F0.shape[1], F1.shape[1])
    np.testing.assert_allclose(Z, g["Z"], atol=1.5e-3, rtol=1e-4)
    np.testing.assert_allclose(np.exp(Z.astype(np.float64)), np.exp(g["Z"].astype(np.float64)), atol=1e-4, rtol=5e-4)
    assert n == len(g["matches"]) >= 80
    np.testing.assert_array_equal(np.array([(q, t) for q, t, _ in ml]), g["matches"])
    np.testing.assert_allclose([d for _, _, d in ml], g["distances"], atol=1e-4, rtol=5e-4)


def test_sg_c1_images_to_matches_fp32(pkg, golden, weight_blobs, sg_c1_blob):
    """Images -> matches on the GPU (fp32): SuperPoint on the C1 stereo images gives the reference
    module's keypoint sets and descriptors, and PointMatching on those features gives the reference's
    matches (compared as keypoint-coordinate pairs: the top-k order of near-equal scores may differ)."""
    from helpers import compare_features
    from rspl_slam_amd import synthetic as SY
    g = golden("sg_c1")
    L, R = SY.stereo_pair(480, 752, seed=int(g["seed"]))
    sp = pkg.SuperPoint(pkg.SuperPointConfig(max_keypoints=400, weights=weight_blobs[0], max_height=480,
                                             max_width=752, max_batch=1))
    assert sp.build(), sp.error
    F = []
    for img, Fr in ((L, g["F0"]), (R, g["F1"])):
        ok, Fg = sp.infer(img)
        assert ok, sp.error
        compare_features(Fg, Fr.astype(np.float64), desc_atol=1e-5, score_atol=1e-5)
        F.append(Fg)
    pm = _pm(pkg, sg_c1_blob, pkg.capi.RSPL_PREC_FP32)
    n, ml = pm.MatchingPoints(F[0], F[1])
    got = {(F[0][1, q], F[0][2, q], F[1][1, t], F[1][2, t]) for q, t, _ in ml}
    F0r, F1r = g["F0"], g["F1"]
    ref = {(F0r[1, q], F0r[2, q], F1r[1, t], F1r[2, t]) for q, t in g["matches"]}
    assert n >= 80 and got == ref


def test_sg_c1_fp16_disagreements_explained(pkg, golden, sg_c1_blob):
    """fp16 (the reference's TensorRT kFP16 engine, super_glue.cpp:132) vs the reference on the C1 pair:
    every match-index disagreement must sit at a near-tie of the reference's own Z within the measured
    fp16 |dZ| (helpers.unexplained_match_disagreements), and the thresholded match agreement is reported."""
    from helpers import unexplained_match_disagreements
    g = golden("sg_c1")
    F0, F1 = g["F0"].astype(np.float64), g["F1"].astype(np.float64)
    G0, G1 = post.normalize_keypoints(F0, 752, 480), post.normalize_keypoints(F1, 752, 480)
    sg = pkg.SuperGlue(pkg.SuperGlueConfig(weights=sg_c1_blob, max_keypoints=400, max_batch=1,
                                           precision=pkg.capi.RSPL_PREC_FP16))
    assert sg.build(), sg.error
    ok, i0, i1, m0, m1 = sg.infer(G0, G1)
    assert ok, sg.error
    Z = sg.debug_scores(0, F0.shape[1], F1.shape[1])
    sig = g["Z"] > np.log(1e-4)
    tol = 2.0 * float(np.abs(Z - g["Z"])[sig].max())  # a disagreement needs a gap below twice the fp16 error
    # and that error itself is bounded absolutely: 0.084 measured on this fixture (round 5), the bound 3x that,
    # so a change that degrades the fp16 path cannot widen the tie margin unnoticed
    assert tol / 2 < 0.25, f"fp16 |dZ| on significant entries {tol / 2:.3g}"
    bad = unexplained_match_disagreements(g["Z"], i0, i1, g["idx0"], g["idx1"], tol)
    agree = ((i0 == g["idx0"]).mean() + (i1 == g["idx1"]).mean()) / 2
    print(f"c1 fp16: index agreement {agree:.4f}, fp16 |dZ| (significant) {tol / 2:.3g}, "
          f"matches {int((i0 >= 0).sum())} vs {int((g['idx0'] >= 0).sum())}, unexplained {bad}")
    assert not bad
