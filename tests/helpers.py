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
