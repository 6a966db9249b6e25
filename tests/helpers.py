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
