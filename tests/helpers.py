"""Shared parity comparators (test infrastructure)."""
import numpy as np


def compare_features(F, G, score_atol=1e-5, desc_atol=1e-5, desc_rtol=1e-3, order_atol=None):
    """Compare two 259 x n feature matrices of the same image.

    Keypoint SET must be identical; columns are matched by (x, y).  Column order must agree except
    that neighbours whose reference scores differ by less than score_atol may be swapped (fp32
    accumulation order vs the reference -- top-k is an ordering by score)."""
    assert F.shape == G.shape, (F.shape, G.shape)
    if F.shape[1] == 0:
        return
    key = lambda M: [(int(x), int(y)) for x, y in zip(M[1], M[2])]
    kf, kg = key(F), key(G)
    assert set(kf) == set(kg), f"keypoint sets differ: {len(set(kf) - set(kg))} extra, {len(set(kg) - set(kf))} missing"
    pos = {k: i for i, k in enumerate(kg)}
    perm = np.array([pos[k] for k in kf])
    Gp = G[:, perm]
    np.testing.assert_allclose(F[0], Gp[0], atol=score_atol, rtol=0)
    np.testing.assert_allclose(F[3:], Gp[3:], atol=desc_atol, rtol=desc_rtol)
    order_atol = score_atol if order_atol is None else order_atol
    moved = np.nonzero(perm != np.arange(len(perm)))[0]
    for i in moved:
        assert abs(G[0, i] - G[0, perm[i]]) < order_atol, f"order differs beyond score tolerance at column {i}"


def unexplained_match_disagreements(Zo, i0, i1, i0r, i1r, tol):
    """Rows / columns whose match index differs from the oracle's and that the oracle's own Z does
    NOT show as a near-tie (indices identical except at ties within the Z tolerance).

    Z is the (N+1) x (M+1) log-assignment of the oracle; decode (src/super_glue.cpp:258-367) can only
    flip where (a) a row or column argmax has a runner-up within tol, or (b) the kept score sits
    within tol of the 0.2 threshold (log space).  Returns the unexplained (kind, index) list."""
    Z = np.asarray(Zo, np.float64)[:-1, :-1]
    N, M = Z.shape
    lthr = np.log(0.2)

    def gap(v):
        if v.size < 2:
            return np.inf
        t = np.partition(v, -2)[-2:]
        return t[1] - t[0]
    rowgap = np.array([gap(Z[i]) for i in range(N)])
    colgap = np.array([gap(Z[:, j]) for j in range(M)])
    amax0, amax1 = Z.argmax(1), Z.argmax(0)

    def row_near(i):
        j = amax0[i]
        return rowgap[i] < tol or colgap[j] < tol or abs(Z[i, j] - lthr) < tol or \
            (i0[i] >= 0 and colgap[i0[i]] < tol) or (i0r[i] >= 0 and colgap[i0r[i]] < tol)

    def col_near(j):
        i = amax1[j]
        return colgap[j] < tol or rowgap[i] < tol or abs(Z[i, j] - lthr) < tol or \
            (i1[j] >= 0 and rowgap[i1[j]] < tol) or (i1r[j] >= 0 and rowgap[i1r[j]] < tol)
    bad = [("row", int(i)) for i in np.nonzero(i0 != i0r)[0] if not row_near(i)]
    bad += [("col", int(j)) for j in np.nonzero(i1 != i1r)[0] if not col_near(j)]
    return bad


def _R_of_q(q):
    """rotation of a unit quaternion (x, y, z, w)"""
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def line_residuals(prob, pose_q, pose_p, lines):
    """Residuals of every line edge at a BA result (EdgeSE3ProjectLine / EdgeStereoSE3ProjectLine,
    edge_project_line.cc:21-42, edge_project_stereo_line.cc:22-51): the quantity the BA minimises
    for a line, independent of the Pluecker coordinates' weakly observed directions."""
    out = []
    for name, sides in (("mono_line", 1), ("stereo_line", 2)):
        d = getattr(prob, name)
        for p, l, c, o in zip(d["pose"], d["lm"], d["cam"], d["obs"]):
            fx, fy, cx, cy, bf = prob.cameras[c]
            Rwc = _R_of_q(pose_q[p] / np.linalg.norm(pose_q[p]))
            Rcw, tcw = Rwc.T, -Rwc.T @ pose_p[p]
            w, dv = lines[l][:3], lines[l][3:]
            for side in range(sides):
                t = tcw.copy()
                if side == 1:
                    t[0] -= bf / fx
                wc = Rcw @ w + np.cross(t, Rcw @ dv)
                l0, l1, l2 = fy * wc[0], fx * wc[1], -fy * cx * wc[0] - fx * cy * wc[1] + fx * fy * wc[2]
                n = np.hypot(l0, l1)
                ob = o[4 * side:4 * side + 4]
                out += [(ob[0] * l0 + ob[1] * l1 + l2) / n, (ob[2] * l0 + ob[3] * l1 + l2) / n]
    return np.array(out)


E2E_CLASSES = ("absent_near_cut", "absent_nms_tie", "competitor_absent", "z_near_tie", "unexplained")


def classify_e2e_disagreements(Fa, Fb, Za, Zb, threshold, score_tol, z_tol, k=400, kp_threshold=0.004,
                               nms_radius=4):
    """End-to-end match disagreements between two front ends on the same image pair, each with its own
    SuperPoint keypoints: path a is the reference (the CPU path), b the one under test.  Fa / Fb = [F0, F1]
    (259 x n feature matrices), Za / Zb their SuperGlue log-assignments.  Matches are decoded from each Z
    (super_glue.cpp:258-367 with `threshold`; point_matching.cc:24-31 mutual re-check) and compared as
    keypoint-coordinate pairs; every match present in one path and not the other is classified:

      absent_near_cut   one of its keypoints is missing from the other path's set and its score is within
                        score_tol of the other path's cut (its k-th score when it kept k, else the 0.004
                        keypoint threshold): the top-k / threshold decision of super_point.cpp:154-204 flips
                        with a score error of that size;
      absent_nms_tie    missing, and the other path keeps a keypoint inside the NMS window (|dx|, |dy| <=
                        nms_radius) whose score is within score_tol (simple_nms picked the other of two
                        near-equal maxima, superpoint.py:16-33);
      competitor_absent all its keypoints are in both sets, but the other path's decision at its row or
                        column goes to a keypoint missing from this path's set (explained by the set change);
      z_near_tie        every keypoint involved is shared and the reference Z shows a near-tie within z_tol:
                        the row / column argmax runner-up, the pair within z_tol of its row or column maximum,
                        the partner's gap, or the threshold (log space);
      unexplained       none of these.
    Returns ({class: count}, [unexplained (side, coords)])."""
    import sys
    import pathlib
    sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "oracle"))
    import post

    def keys(F):
        return {(int(x), int(y)): i for i, (x, y) in enumerate(zip(F[1], F[2]))}

    def matches(F, Z):
        m, _ = post.match_points(*post.decode(Z, threshold=threshold))
        return {(int(F[0][1, q]), int(F[0][2, q]), int(F[1][1, t]), int(F[1][2, t])) for q, t in m}, m

    ka, kb = [keys(F) for F in Fa], [keys(F) for F in Fb]
    ma, _ = matches(Fa, Za)
    mb, _ = matches(Fb, Zb)
    # each path's decision per keypoint: row -> column keypoint, column -> row keypoint (mutual NN argmax)
    def argmaxes(F, Z):
        S = np.asarray(Z, np.float64)[:-1, :-1]
        if S.size == 0:
            return {}, {}
        r = {(int(F[0][1, i]), int(F[0][2, i])): (int(F[1][1, j]), int(F[1][2, j])) for i, j in enumerate(S.argmax(1))}
        c = {(int(F[1][1, j]), int(F[1][2, j])): (int(F[0][1, i]), int(F[0][2, i])) for j, i in enumerate(S.argmax(0))}
        return r, c
    arg = {"a": argmaxes(Fa, Za), "b": argmaxes(Fb, Zb)}
    S = np.asarray(Za, np.float64)[:-1, :-1]
    lthr = np.log(threshold) if threshold > 0 else -np.inf

    def gap(v):
        if v.size < 2:
            return np.inf
        t = np.partition(v, -2)[-2:]
        return t[1] - t[0]

    def cut(F):
        return float(F[0].min()) if F.shape[1] >= k else kp_threshold

    def absent_class(p, img, own, other):
        """keypoint p (coords) of image img kept by path `own`, missing from path `other`"""
        Fo, Ft = (Fa, Fb) if own == "a" else (Fb, Fa)
        ko = (ka if own == "a" else kb)[img]
        s = float(Fo[img][0, ko[p]])
        if s - cut(Ft[img]) <= score_tol:
            return "absent_near_cut"
        kt = kb[img] if own == "a" else ka[img]
        for q, i in kt.items():
            if abs(q[0] - p[0]) <= nms_radius and abs(q[1] - p[1]) <= nms_radius and \
                    abs(float(Ft[img][0, i]) - s) <= score_tol:
                return "absent_nms_tie"
        return None

    def z_tie(p0, p1):
        if S.size == 0:
            return False
        r, c = ka[0][p0], ka[1][p1]
        row, col = S[r], S[:, c]
        if gap(row) < z_tol or gap(col) < z_tol or row.max() - S[r, c] < z_tol or col.max() - S[r, c] < z_tol:
            return True
        if abs(S[r, c] - lthr) < z_tol:
            return True
        return gap(S[:, int(row.argmax())]) < z_tol or gap(S[int(col.argmax())]) < z_tol

    counts = {c: 0 for c in E2E_CLASSES}
    bad = []
    for side, mine, other_set, own, oth in (("a_only", ma, mb, "a", "b"), ("b_only", mb, ma, "b", "a")):
        ko_other = kb if own == "a" else ka
        for m in sorted(mine - other_set):
            p0, p1 = m[:2], m[2:]
            cls = None
            for img, p in ((0, p0), (1, p1)):
                if p not in ko_other[img]:
                    cls = absent_class(p, img, own, oth) or "unexplained"
                    break
            if cls is None:
                # the other path's decision at this row / column: to a keypoint this path lacks?
                r_oth, c_oth = arg[oth]
                kown = ka if own == "a" else kb
                comp = [r_oth.get(p0), c_oth.get(p1)]
                if (comp[0] is not None and comp[0] not in kown[1]) or (comp[1] is not None and comp[1] not in kown[0]):
                    cls = "competitor_absent"
                elif p0 in ka[0] and p1 in ka[1] and z_tie(p0, p1):
                    cls = "z_near_tie"
                else:
                    cls = "unexplained"
            counts[cls] += 1
            if cls == "unexplained":
                bad.append((side, m))
    return counts, bad
