"""BASELINE C1 plumbing (configs[0]: "first 100 stereo pairs, SuperPoint/SuperGlue + host g2o, plumbing"):
100 synthetic EuRoC-shaped stereo pairs (480x752 u8, seeded textured scenes; EuRoC images are not in
the container) through the keyframe front end twice, and the two compared pair by pair --

  (a) the CPU path: the oracle's C restatement of SuperPoint (convert2onnx/superpoint.py + the
      host post-processing of super_point.cpp:154-319) on the left and right image, SuperGlue on
      (left, right) (superglue.py + super_glue.cpp decode), PointMatching's mutual re-check
      (point_matching.cc:12-48), and the line part of Frame::AddRightFeatures (frame.cc:150-203:
      disparity filter, AssignPointsToLines x2, MatchLines, right line per left line) restated in
      oracle/lines_ref.py, on one frame's FLD-like segments merged by LineDetector (lines_ref);
  (b) librspl: SuperPoint, PointMatching and the stereo line association on the GPU (fp32 parity
      path), the merge passes in native C++ -- and the fp16 (TensorRT kFP16-equivalent) front end.

Per pair it records keypoint agreement, descriptor error, the log-assignment Z error, match agreement
(fp32 and fp16) and the agreement of the stereo line association.  The weights are seeded synthetic
ones (no trained weights exist here): SuperPoint's default profile, and SuperGlue's "c1" profile
(weights.SG_WEIGHT_GAIN_C1), under which 25-38 % of the keypoints are matched above the reference's
0.2 threshold (super_glue.cpp:355) -- so the thresholded decode and the DMatch distances are compared
pair by pair (the default profile left every probability below 0.2 here).  The mutual nearest
neighbours of Z with the threshold at 0 are compared too, and feed the stereo line association.
fp16 (the TensorRT kFP16 analogue) is checked twice: fp16 SuperGlue on the CPU path's features (every
index disagreement must sit at a near-tie of the CPU Z within twice the measured fp16 |dZ|:
helpers.unexplained_match_disagreements), and fp16 SuperPoint + SuperGlue end to end (keypoint overlap
per image, match agreement by coordinates).  MapBuilder / tracking are not built (out of scope); the
map-side BA over a 100-keyframe sequence is tools/run_sequence.py.  Prints one JSON line; per-pair
records go to --out."""
import argparse
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()
pkg.capi.load()
from helpers import E2E_CLASSES, classify_e2e_disagreements, unexplained_match_disagreements  # noqa: E402
import lines_ref as LR  # noqa: E402  (the CPU path being compared against; test infrastructure)
import oracle  # noqa: E402
import post  # noqa: E402

H, W, K = 480, 752, 400
DISP = 12  # synthetic.stereo_pair's default disparity


def key_index(F):
    return {(int(x), int(y)): i for i, (x, y) in enumerate(zip(F[1], F[2]))}


def match_set(m):
    return {(int(q), int(t)) for q, t in np.asarray(m).reshape(-1, 2)}


def match_coords(m, F0, F1):
    """matches as keypoint-coordinate pairs: comparable across paths whose keypoint lists differ"""
    return {(int(F0[1, q]), int(F0[2, q]), int(F1[1, t]), int(F1[2, t])) for q, t in np.asarray(m).reshape(-1, 2)}


def align_z(Zg, Fg0, Fg1, Fc0, Fc1):
    """Zg with its rows / columns put in the CPU path's keypoint order (the dustbin row / column last),
    or None when the keypoint sets differ.  fp32 scores that differ in the last bits can swap the
    top-k order of near-equal scores (std::sort by score, super_point.cpp:154-204) while the sets
    agree; SuperGlue is permutation-equivariant, so Z is compared in one order."""
    kg0, kg1 = key_index(Fg0), key_index(Fg1)
    c0 = [(int(x), int(y)) for x, y in zip(Fc0[1], Fc0[2])]
    c1 = [(int(x), int(y)) for x, y in zip(Fc1[1], Fc1[2])]
    if set(c0) != set(kg0) or set(c1) != set(kg1):
        return None
    rows = [kg0[c] for c in c0] + [len(c0)]
    cols = [kg1[c] for c in c1] + [len(c1)]
    return Zg[np.ix_(rows, cols)]


def shared_z(Zg, Fg0, Fg1, Zc, Fc0, Fc1):
    """Zg and Zc restricted to the keypoints both paths kept (rows / columns in the CPU path's order, the
    dustbin row / column last): comparable whatever the two keypoint sets are (with different sets the
    difference includes the effect of the keypoints only one path has -- attention and Sinkhorn see all)."""
    kg0, kg1 = key_index(Fg0), key_index(Fg1)
    c0 = [(int(x), int(y)) for x, y in zip(Fc0[1], Fc0[2])]
    c1 = [(int(x), int(y)) for x, y in zip(Fc1[1], Fc1[2])]
    rc = [i for i, c in enumerate(c0) if c in kg0] + [len(c0)]
    cc = [j for j, c in enumerate(c1) if c in kg1] + [len(c1)]
    rg = [kg0[c0[i]] for i in rc[:-1]] + [Fg0.shape[1]]
    cg = [kg1[c1[j]] for j in cc[:-1]] + [Fg1.shape[1]]
    return Zg[np.ix_(rg, cg)], Zc[np.ix_(rc, cc)]


def score_error(Fa, Fb):
    """max |score| difference over the keypoints both paths kept, both images"""
    e = 0.0
    for A, B in zip(Fa, Fb):
        ka, kb = key_index(A), key_index(B)
        for c in set(ka) & set(kb):
            e = max(e, abs(float(A[0, ka[c]]) - float(B[0, kb[c]])))
    return e


def e2e(Fc, Z, Fg, Zg):
    """end-to-end disagreements of the GPU path (its own keypoints, its Z) vs the CPU path, thresholded
    (0.2, the reference's decode) and mutual-NN (threshold 0), classified (helpers.classify_e2e_disagreements)
    with the pair's own measured errors as the tie margins: 2x the score error on the shared keypoints and 2x
    the significant-entry |dZ| on them (floors 1e-7 / 1e-6)"""
    zg, zc = shared_z(Zg, Fg[0], Fg[1], Z, Fc[0], Fc[1])
    sig = zc > np.log(1e-4)
    dz = float(np.abs(zg - zc)[sig].max()) if sig.any() else 0.0
    s_tol = max(2.0 * score_error(Fc, Fg), 1e-7)
    z_tol = max(2.0 * dz, 1e-6)
    out = {"score_tol": s_tol, "z_tol": z_tol}
    for name, thr in (("thresholded", 0.2), ("mutual_nn", 0.0)):
        cnt, bad = classify_e2e_disagreements(Fc, Fg, Z, Zg, thr, s_tol, z_tol, k=K)
        out[name] = cnt
        out[name + "_unexplained"] = [list(map(int, m)) for _, m in bad][:8]
    return out


def e2e_fp16_decomposed(F16, Z16g, Fc, Z, sg_w):
    """Every end-to-end fp16 match disagreement (fp16 SuperPoint + fp16 SuperGlue vs the CPU path), split by
    cause with the reference's own fp32 SuperGlue run on the fp16 SuperPoint features (Z16c):
      fp16_superpoint_input    the fp32 SuperGlue makes the GPU's decision on those features too: the fp16
                               SuperPoint outputs (scores, descriptors, a keypoint at the top-k cut) changed
                               SuperGlue's input, the reference algorithm does the same on that input;
      fp16_superglue_near_tie  the GPU fp16 SuperGlue and the fp32 one disagree on the same features, and Z16c
                               shows a near-tie within 2x the pair's fp16 SuperGlue |dZ| (significant entries);
      unexplained              neither."""
    g0, g1 = post.normalize_keypoints(F16[0], W, H), post.normalize_keypoints(F16[1], W, H)
    Z16c = oracle.sg_forward(sg_w, *post.sg_inputs(g0), *post.sg_inputs(g1))
    sig = Z16c > np.log(1e-4)
    dz = float(np.abs(Z16g - Z16c)[sig].max()) if sig.any() else 0.0
    out = {"sg_only_dZ_sig": dz}
    for name, thr in (("thresholded", 0.2), ("mutual_nn", 0.0)):
        dg, dcc, dc = post.decode(Z16g, threshold=thr), post.decode(Z16c, threshold=thr), post.decode(Z, threshold=thr)
        mg = match_coords(post.match_points(*dg)[0], F16[0], F16[1])
        m16c = match_coords(post.match_points(*dcc)[0], F16[0], F16[1])
        mc = match_coords(post.match_points(*dc)[0], Fc[0], Fc[1])
        bad_sg = {(int(F16[0][1, i]), int(F16[0][2, i])) for kind, i in
                  unexplained_match_disagreements(Z16c, dg[0], dg[1], dcc[0], dcc[1], 2.0 * dz) if kind == "row"}
        bad_sg |= {("col", int(F16[1][1, j]), int(F16[1][2, j])) for kind, j in
                   unexplained_match_disagreements(Z16c, dg[0], dg[1], dcc[0], dcc[1], 2.0 * dz) if kind == "col"}
        cnt = {"fp16_superpoint_input": 0, "fp16_superglue_near_tie": 0, "unexplained": 0}
        for m in (mc ^ mg):
            if (m in mg) == (m in m16c):
                cnt["fp16_superpoint_input"] += 1
            elif (m[0], m[1]) in bad_sg or ("col", m[2], m[3]) in bad_sg:
                cnt["unexplained"] += 1
            else:
                cnt["fp16_superglue_near_tie"] += 1
        out[name] = cnt
    return out


def z_errors(Zg, Z):
    """max |exp(Zg) - exp(Z)| (assignment probabilities) and max |dZ| where the CPU probability >= 1e-4;
    log-probabilities far below that amplify rounding and carry no decision"""
    if Zg.shape != Z.shape:
        return float("nan"), float("nan")
    dp = float(np.abs(np.exp(Zg.astype(np.float64)) - np.exp(Z.astype(np.float64))).max())
    sig = Z > np.log(1e-4)
    dz = float(np.abs(Zg - Z)[sig].max()) if sig.any() else 0.0
    return dp, dz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=100)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default="gpurun_out/c1_pairs.jsonl")
    a = ap.parse_args()
    oracle.set_threads(a.threads)
    sp_w, _ = pkg.weights.ensure_blobs(str(ROOT / "weights"))
    sg_w = pkg.weights.ensure_sg_profile_blob(str(ROOT / "weights"), "c1")
    bf = pkg.synthetic.EUROC_BF
    lim = (bf / 10.0, bf / 0.1, 2.0)  # MinXDiff, MaxXDiff, MaxYDiff (camera.cc:21-22)
    C = pkg.capi
    sps, pms = {}, {}
    for name, prec in (("fp32", C.RSPL_PREC_FP32), ("fp16", C.RSPL_PREC_FP16)):
        sps[name] = pkg.SuperPoint(pkg.SuperPointConfig(max_keypoints=K, weights=sp_w, max_height=H, max_width=W,
                                                        max_batch=1, precision=prec))
        assert sps[name].build(), sps[name].error
        pms[name] = pkg.PointMatching(pkg.SuperGlueConfig(image_width=W, image_height=H, weights=sg_w,
                                                          max_keypoints=K, max_batch=1, precision=prec))
    # split-fp16 SuperPoint (RSPL_PREC_FP16X3) in front of the fp16 SuperGlue
    sps["fp16x3"] = pkg.SuperPoint(pkg.SuperPointConfig(max_keypoints=K, weights=sp_w, max_height=H, max_width=W,
                                                        max_batch=1, precision=C.RSPL_PREC_FP16X3))
    assert sps["fp16x3"].build(), sps["fp16x3"].error
    pms["fp16x3"] = pms["fp16"]
    lm = pkg.lines.LineMatcher(max_lines=512, max_points=512)
    out = pathlib.Path(a.out)
    out.parent.mkdir(parents=True, exist_ok=True)
    rows, t_cpu, t_gpu = [], 0.0, 0.0
    with out.open("w") as fo:
        for t in range(a.pairs):
            L, R = pkg.synthetic.stereo_pair(H, W, seed=300 + t)
            sc = pkg.synthetic.line_scene(n_lines=80, n_points=16, seed=300 + t, width=W, height=H)
            # (a) CPU path
            t0 = time.perf_counter()
            Fc = []
            for img in (L, R):
                s, d = oracle.sp_forward(sp_w, post.image_to_input(img))
                Fc.append(post.sp_postprocess(s, d, 0.004, 4, K))
            g0, g1 = post.normalize_keypoints(Fc[0], W, H), post.normalize_keypoints(Fc[1], W, H)
            Z = oracle.sg_forward(sg_w, *post.sg_inputs(g0), *post.sg_inputs(g1))
            mc, _ = post.match_points(*post.decode(Z))
            nnc, _ = post.match_points(*post.decode(Z, threshold=0.0))  # mutual NN, no threshold
            l0c, l1c = LR.line_extractor(sc["seg_left"]), LR.line_extractor(sc["seg_right"])
            km = LR.stereo_filter(Fc[0][1], Fc[1][1], Fc[0][2], Fc[1][2], nnc, *lim)
            r0, r1 = LR.assign_points_to_lines(l0c, Fc[0][1:3].T), LR.assign_points_to_lines(l1c, Fc[1][1:3].T)
            lrc, lvc = LR.right_lines(l1c, LR.match_lines(r0, r1, km, Fc[0].shape[1], Fc[1].shape[1]), len(l0c))
            t_cpu += time.perf_counter() - t0
            # (b) GPU path, fp32 (parity) and fp16
            res = {}
            for name in ("fp32", "fp16", "fp16x3"):
                t0 = time.perf_counter()
                Fg = []
                for img in (L, R):
                    ok, F = sps[name].infer(img)
                    assert ok, sps[name].error
                    Fg.append(F)
                nm, ml = pms[name].MatchingPoints(Fg[0], Fg[1])
                mg = np.array([(q, tt) for q, tt, _ in ml], np.int32).reshape(-1, 2)
                Zg = pms[name].superglue.debug_scores(0, Fg[0].shape[1], Fg[1].shape[1])
                nng, _ = post.match_points(*post.decode(Zg, threshold=0.0))
                l0g, l1g = pkg.lines.LineExtractor(sc["seg_left"]), pkg.lines.LineExtractor(sc["seg_right"])
                lrg, lvg, kept = lm.StereoLines(l0g, Fg[0], l1g, Fg[1], nng, lim)
                if name == "fp32":
                    t_gpu += time.perf_counter() - t0
                res[name] = (Fg, mg, nng, Zg, l0g, lrg, lvg)
            # fp16 SuperGlue on the CPU path's own features: its disagreements vs the CPU Z must be near-ties
            n16, ml16 = pms["fp16"].MatchingPoints(Fc[0], Fc[1])
            Z16 = pms["fp16"].superglue.debug_scores(0, Fc[0].shape[1], Fc[1].shape[1])
            d16 = post.decode(Z16)
            dc = post.decode(Z)
            sig = Z > np.log(1e-4)
            dz16 = float(np.abs(Z16 - Z)[sig].max()) if sig.any() else 0.0
            bad16 = unexplained_match_disagreements(Z, d16[0], d16[1], dc[0], dc[1], 2.0 * dz16)
            agree16_idx = float(((d16[0] == dc[0]).mean() + (d16[1] == dc[1]).mean()) / 2)
            m16 = match_set(np.array([(q, tt) for q, tt, _ in ml16], np.int32).reshape(-1, 2))
            Fg, mg, nng, Zg, l0g, lrg, lvg = res["fp32"]
            kc, kg = key_index(Fc[0]), key_index(Fg[0])
            common = sorted(set(kc) & set(kg))
            dmax = max(float(np.abs(Fg[0][3:, kg[c]] - Fc[0][3:, kc[c]]).max()) for c in common) if common else 0.0
            sc_, sg_ = match_set(mc), match_set(mg)
            nc_, ng_ = match_set(nnc), match_set(nng)
            cc_ = match_coords(nnc, Fc[0], Fc[1])
            cg_ = match_coords(nng, Fg[0], Fg[1])
            F16 = res["fp16"][0]
            c16 = match_coords(res["fp16"][2], F16[0], F16[1])
            za = align_z(Zg, Fg[0], Fg[1], Fc[0], Fc[1])
            za16 = align_z(res["fp16"][3], F16[0], F16[1], Fc[0], Fc[1])
            # every pair: Z on the keypoints both paths kept (the sets may differ)
            zs32 = shared_z(Zg, Fg[0], Fg[1], Z, Fc[0], Fc[1])
            zs16 = shared_z(res["fp16"][3], F16[0], F16[1], Z, Fc[0], Fc[1])
            dps32, _ = z_errors(*zs32)
            dps16, dzs16 = z_errors(*zs16)
            e32, e16 = e2e(Fc, Z, Fg, Zg), e2e(Fc, Z, F16, res["fp16"][3])
            e16d = e2e_fp16_decomposed(F16, res["fp16"][3], Fc, Z, sg_w)
            zerr = float(np.abs(za - Z).max()) if za is not None else float("nan")
            # fp32 thresholded-decode disagreements (GPU Z in the CPU order) must be near-ties of the CPU Z
            bad32 = -1
            if za is not None:
                sig32 = Z > np.log(1e-4)
                dz32 = float(np.abs(za - Z)[sig32].max()) if sig32.any() else 0.0
                da = post.decode(za)
                bad32 = len(unexplained_match_disagreements(Z, da[0], da[1], dc[0], dc[1], 2.0 * dz32))
            dp, dzs = z_errors(za, Z) if za is not None else (float("nan"), float("nan"))
            dp16, _ = z_errors(za16, Z) if za16 is not None else (float("nan"), float("nan"))
            order_same = all(np.array_equal(Fg[i][1:3], Fc[i][1:3]) for i in (0, 1) if Fg[i].shape == Fc[i].shape)
            lines_same = l0g.shape == l0c.shape and bool(np.array_equal(l0g, l0c))
            F16e = res["fp16"][0]
            overlap16 = [len(set(key_index(F16e[i])) & set(key_index(Fc[i]))) / max(1, Fc[i].shape[1]) for i in (0, 1)]
            F3 = res["fp16x3"][0]
            c3 = match_coords(res["fp16x3"][2], F3[0], F3[1])
            m3 = match_coords(res["fp16x3"][1], F3[0], F3[1])
            overlap3 = [len(set(key_index(F3[i])) & set(key_index(Fc[i]))) / max(1, Fc[i].shape[1]) for i in (0, 1)]
            e3 = e2e(Fc, Z, F3, res["fp16x3"][3])
            desc3 = max((float(np.abs(F3[i][3:, key_index(F3[i])[c]] - Fc[i][3:, key_index(Fc[i])[c]]).max())
                         for i in (0, 1) for c in set(key_index(F3[i])) & set(key_index(Fc[i]))), default=0.0)
            dist_c = {(int(q), int(tt)): d for (q, tt), d in zip(np.asarray(mc).reshape(-1, 2), post.match_points(*dc)[1])}
            dist_g = {(int(q), int(tt)): d for q, tt, d in pms["fp32"].MatchingPoints(Fg[0], Fg[1])[1]}
            dist_err = max((abs(dist_c[k] - dist_g[k]) for k in dist_c if k in dist_g), default=0.0)
            # geometry: stereo_pair's right view is the left texture shifted by +DISP px (plus sensor
            # noise), so keypoint (x, y) of the left image sits at (x + DISP, y) in the right one
            kl, kr = Fc[0][1:3].T, Fc[1][1:3].T
            rep = float(np.mean([np.hypot(kr[:, 0] - (x + DISP), kr[:, 1] - y).min() <= 2.0 for x, y in kl])) \
                if len(kl) and len(kr) else 0.0
            mcc = np.asarray(mc).reshape(-1, 2)
            geo = int(np.sum((np.abs(Fc[1][1, mcc[:, 1]] - Fc[0][1, mcc[:, 0]] - DISP) <= 2.0) &
                             (np.abs(Fc[1][2, mcc[:, 1]] - Fc[0][2, mcc[:, 0]]) <= 2.0))) if len(mcc) else 0
            row = {"pair": t,
                   "keypoint_repeatability_cpu": rep, "thresholded_matches_geometric_cpu": geo,
                   "keypoints": [int(Fc[0].shape[1]), int(Fc[1].shape[1])],
                   "keypoint_sets_identical": bool(set(kc) == set(kg)) and
                   set(key_index(Fc[1])) == set(key_index(Fg[1])),
                   "keypoint_order_identical": bool(order_same and all(Fg[i].shape == Fc[i].shape for i in (0, 1))),
                   "desc_max_abs_diff": dmax,
                   "Z_max_abs_diff_fp32": zerr,
                   "P_max_abs_diff_fp32": dp, "Z_sig_max_abs_diff_fp32": dzs, "P_max_abs_diff_fp16_same_set": dp16,
                   "P_max_abs_diff_fp32_shared": dps32, "P_max_abs_diff_fp16": dps16, "Z_sig_max_abs_diff_fp16": dzs16,
                   "e2e_fp32": e32, "e2e_fp16": e16, "e2e_fp16_by_cause": e16d,
                   "matches_cpu": len(sc_), "matches_gpu_fp32": len(sg_), "matches_identical": sc_ == sg_,
                   "matches_identical_coords": match_coords(mc, Fc[0], Fc[1]) == match_coords(mg, Fg[0], Fg[1]),
                   "match_distance_max_abs_diff_fp32": float(dist_err),
                   "unexplained_disagreements_fp32": bad32,
                   "sg16_on_cpu_features": {"matches": int(n16), "matches_identical": m16 == sc_,
                                            "index_agreement": agree16_idx, "dZ_sig_max": dz16,
                                            "unexplained_disagreements": len(bad16)},
                   "keypoint_overlap_fp16": overlap16,
                   "mutual_nn_cpu": len(nc_),
                   "match_agreement_fp32": len(nc_ & ng_) / max(1, len(nc_ | ng_)),
                   "match_agreement_fp32_coords": len(cc_ & cg_) / max(1, len(cc_ | cg_)),
                   "match_agreement_fp16": len(cc_ & c16) / max(1, len(cc_ | c16)),
                   "keypoint_sets_identical_fp16": set(key_index(Fc[0])) == set(key_index(F16[0])) and
                   set(key_index(Fc[1])) == set(key_index(F16[1])),
                   "keypoint_overlap_fp16x3": overlap3,
                   "keypoint_sets_identical_fp16x3": all(set(key_index(Fc[i])) == set(key_index(F3[i])) for i in (0, 1)),
                   "desc_max_abs_diff_fp16x3": desc3,
                   "match_agreement_fp16x3": len(cc_ & c3) / max(1, len(cc_ | c3)),
                   "thresholded_matches_identical_coords_fp16x3": m3 == match_coords(mc, Fc[0], Fc[1]),
                   "e2e_fp16x3": e3,
                   "lines_left": int(len(l0c)), "merged_lines_identical": lines_same,
                   "right_lines_valid_cpu": int(lvc.sum()), "right_lines_valid_gpu": int(lvg.sum()),
                   "line_association_identical": lines_same and bool(np.array_equal(lvc, lvg)) and
                   bool(np.array_equal(lrc[lvc], lrg[lvg]))}
            rows.append(row)
            fo.write(json.dumps(row) + "\n")
            if t % 10 == 0:
                print(f"pair {t}: mutual NN cpu {len(nc_)} gpu {len(ng_)} agreement {row['match_agreement_fp32']:.4f}"
                      f" fp16 {row['match_agreement_fp16']:.4f} |dZ| {zerr:.2e} |dP| {dp:.2e} |dP16| {dp16:.2e}", file=sys.stderr, flush=True)
    agg = lambda k: float(np.mean([r[k] for r in rows]))
    print(json.dumps({
        "pairs": len(rows), "image": f"{W}x{H}", "max_keypoints": K,
        "keypoint_sets_identical_frac": agg("keypoint_sets_identical"),
        "desc_max_abs_diff": float(max(r["desc_max_abs_diff"] for r in rows)),
        "keypoint_order_identical_frac": agg("keypoint_order_identical"),
        # Z / P over the pairs whose keypoint sets agree, in the CPU path's keypoint order (align_z)
        "Z_max_abs_diff_fp32": float(np.nanmax([r["Z_max_abs_diff_fp32"] for r in rows])),
        "P_max_abs_diff_fp32": float(np.nanmax([r["P_max_abs_diff_fp32"] for r in rows])),
        "Z_sig_max_abs_diff_fp32": float(np.nanmax([r["Z_sig_max_abs_diff_fp32"] for r in rows])),
        # fp16 end to end (fp16 SuperPoint + SuperGlue): Z on the keypoints both paths kept, every pair
        "P_max_abs_diff_fp16": float(np.nanmax([r["P_max_abs_diff_fp16"] for r in rows])),
        "P_max_abs_diff_fp16_pairs": int(sum(np.isfinite(r["P_max_abs_diff_fp16"]) for r in rows)),
        "P_max_abs_diff_fp16_p50": float(np.nanmedian([r["P_max_abs_diff_fp16"] for r in rows])),
        "Z_sig_max_abs_diff_fp16": float(np.nanmax([r["Z_sig_max_abs_diff_fp16"] for r in rows])),
        "P_max_abs_diff_fp16_same_set_pairs": int(sum(np.isfinite(r["P_max_abs_diff_fp16_same_set"]) for r in rows)),
        "P_max_abs_diff_fp32_shared": float(np.nanmax([r["P_max_abs_diff_fp32_shared"] for r in rows])),
        # every end-to-end match disagreement (matches as keypoint-coordinate pairs, each path with its own
        # keypoints), classified: keypoint absent near the top-k cut / at an NMS near-tie, decision going to a
        # keypoint the other path lacks, near-tie of the CPU Z, or unexplained (helpers.classify_e2e_disagreements)
        **{f"e2e_{p}_{kind}": {c: int(sum(r[f"e2e_{p}"][kind][c] for r in rows)) for c in E2E_CLASSES}
           for p in ("fp32", "fp16") for kind in ("thresholded", "mutual_nn")},
        # the same disagreements split by cause (e2e_fp16_decomposed: the reference's fp32 SuperGlue re-run on the
        # fp16 SuperPoint features separates the SuperPoint input change from SuperGlue's own fp16 rounding)
        **{f"e2e_fp16_by_cause_{kind}": {c: int(sum(r["e2e_fp16_by_cause"][kind][c] for r in rows))
                                         for c in ("fp16_superpoint_input", "fp16_superglue_near_tie", "unexplained")}
           for kind in ("thresholded", "mutual_nn")},
        "sg_only_fp16_dZ_sig_max": float(max(r["e2e_fp16_by_cause"]["sg_only_dZ_sig"] for r in rows)),
        "unexplained_end_to_end_fp16": int(sum(r["e2e_fp16_by_cause"][k]["unexplained"] for r in rows
                                               for k in ("thresholded", "mutual_nn"))),
        "unexplained_end_to_end_fp16_self_calibrated_classes": int(sum(r["e2e_fp16"][k]["unexplained"] for r in rows
                                                                       for k in ("thresholded", "mutual_nn"))),
        "unexplained_end_to_end_fp32": int(sum(r["e2e_fp32"][k]["unexplained"] for r in rows
                                               for k in ("thresholded", "mutual_nn"))),
        "thresholded_matches_coords_differ_pairs_fp32": [r["pair"] for r in rows if not r["matches_identical_coords"]],
        "keypoint_sets_identical_fp16_frac": agg("keypoint_sets_identical_fp16"),
        "thresholded_matches_identical_frac": agg("matches_identical"),
        "thresholded_matches_identical_coords_frac": agg("matches_identical_coords"),
        "match_distance_max_abs_diff_fp32": float(max(r["match_distance_max_abs_diff_fp32"] for r in rows)),
        # pairs whose keypoint sets agree: decode disagreements of the fp32 GPU Z that the CPU Z does not show as
        # a near-tie (argmax runner-up or the 0.2 threshold within 2x the pair's fp32 |dZ|)
        "unexplained_disagreements_fp32_total": int(sum(max(r["unexplained_disagreements_fp32"], 0) for r in rows)),
        "pairs_compared_fp32": int(sum(r["unexplained_disagreements_fp32"] >= 0 for r in rows)),
        "matches_per_pair_cpu": agg("matches_cpu"),
        "matches_per_pair_min_cpu": int(min(r["matches_cpu"] for r in rows)),
        # the seeded (untrained) networks: how many keypoints repeat under the pair's pure +DISP px shift,
        # and how many thresholded matches are geometrically right -- the C1 record is plumbing (the
        # same bytes through two implementations), not a tracking-quality measurement
        "keypoint_repeatability_cpu_mean": agg("keypoint_repeatability_cpu"),
        "thresholded_matches_geometric_frac_cpu": float(sum(r["thresholded_matches_geometric_cpu"] for r in rows) /
                                                       max(1, sum(r["matches_cpu"] for r in rows))),
        "sg_fp16_on_cpu_features": {
            "index_agreement_mean": float(np.mean([r["sg16_on_cpu_features"]["index_agreement"] for r in rows])),
            "index_agreement_min": float(min(r["sg16_on_cpu_features"]["index_agreement"] for r in rows)),
            "thresholded_matches_identical_frac": float(np.mean([r["sg16_on_cpu_features"]["matches_identical"]
                                                                 for r in rows])),
            "dZ_sig_max": float(max(r["sg16_on_cpu_features"]["dZ_sig_max"] for r in rows)),
            "unexplained_disagreements_total": int(sum(r["sg16_on_cpu_features"]["unexplained_disagreements"]
                                                       for r in rows)),
            "note": "fp16 SuperGlue on the CPU path's features vs the CPU Z; a disagreement is explained when the "
                    "CPU Z shows a near-tie (argmax runner-up or the 0.2 threshold) within 2x the pair's fp16 |dZ|"},
        "keypoint_overlap_fp16_mean": float(np.mean([np.mean(r["keypoint_overlap_fp16"]) for r in rows])),
        "keypoint_overlap_fp16_min": float(min(min(r["keypoint_overlap_fp16"]) for r in rows)),
        "mutual_nn_per_pair_cpu": agg("mutual_nn_cpu"),
        "match_agreement_fp32_mean": agg("match_agreement_fp32"),
        "match_agreement_fp32_min": float(min(r["match_agreement_fp32"] for r in rows)),
        "match_agreement_fp32_coords_mean": agg("match_agreement_fp32_coords"),
        "match_agreement_fp16_mean": agg("match_agreement_fp16"),
        "match_agreement_fp16_min": float(min(r["match_agreement_fp16"] for r in rows)),
        # split-fp16 SuperPoint (RSPL_PREC_FP16X3: hi + lo operands, three fp16 MFMA products) + fp16 SuperGlue
        "fp16x3": {
            "keypoint_overlap_min": float(min(min(r["keypoint_overlap_fp16x3"]) for r in rows)),
            "keypoint_overlap_mean": float(np.mean([np.mean(r["keypoint_overlap_fp16x3"]) for r in rows])),
            "keypoint_sets_identical_frac": agg("keypoint_sets_identical_fp16x3"),
            "desc_max_abs_diff": float(max(r["desc_max_abs_diff_fp16x3"] for r in rows)),
            "match_agreement_mean": agg("match_agreement_fp16x3"),
            "match_agreement_min": float(min(r["match_agreement_fp16x3"] for r in rows)),
            "thresholded_matches_identical_coords_frac": agg("thresholded_matches_identical_coords_fp16x3"),
            **{f"e2e_{kind}": {c: int(sum(r["e2e_fp16x3"][kind][c] for r in rows)) for c in E2E_CLASSES}
               for kind in ("thresholded", "mutual_nn")},
            "note": "SuperPoint in split fp16 (RSPL_PREC_FP16X3), SuperGlue fp16; vs the CPU path by keypoint "
                    "coordinates; the remaining disagreements are the fp16 SuperGlue's, classified as for fp32"},
        "line_association_identical_frac": agg("line_association_identical"),
        "right_lines_valid_per_pair": agg("right_lines_valid_cpu"),
        "cpu_s_per_pair": round(t_cpu / len(rows), 3), "cpu_threads": a.threads,
        "gpu_fp32_host_api_s_per_pair": round(t_gpu / len(rows), 4),
        "weights": "SuperPoint seeded default profile; SuperGlue seeded 'c1' profile (weights.SG_WEIGHT_GAIN_C1)",
        "note": "synthetic stereo pairs (EuRoC absent); the CPU path is the oracle restatement of the "
                "reference's SP/SG modules + host code; GPU = librspl through its host-array API"}))


if __name__ == "__main__":
    main()
