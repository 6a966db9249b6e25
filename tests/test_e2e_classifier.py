"""The end-to-end match-disagreement classifier (helpers.classify_e2e_disagreements) used by the C1 record and
the fp16 parity tests, on CPU: two front ends on the reference's own fixture pair whose keypoint sets differ in
one keypoint at the top-k cut."""
import numpy as np

import oracle
import post
from helpers import E2E_CLASSES, classify_e2e_disagreements


def _sg(sg_w, Fa, Fb):
    ga, gb = post.normalize_keypoints(Fa, 752, 480), post.normalize_keypoints(Fb, 752, 480)
    return oracle.sg_forward(sg_w, *post.sg_inputs(ga), *post.sg_inputs(gb))


def test_classifier_identical_and_cut_swap(golden, sg_c1_blob):
    g = golden("sg_c1")
    F0, F1 = g["F0"].astype(np.float64)[:, :120], g["F1"].astype(np.float64)[:, :121]
    Z = _sg(sg_c1_blob, F0, F1)
    counts, bad = classify_e2e_disagreements([F0, F1], [F0, F1], Z, Z, 0.2, 1e-7, 1e-6, k=120)
    assert sum(counts.values()) == 0 and not bad
    # path b kept the (n+1)-th keypoint of image 1 instead of the n-th (a swap at the top-k cut), n chosen so
    # that path a matches its n-th keypoint
    for n in range(120, 60, -1):
        F1a = F1[:, :n]
        Za = _sg(sg_c1_blob, F0, F1a)
        if post.decode(Za, threshold=0.0)[1][n - 1] >= 0:
            break
    F1b = np.concatenate([F1[:, :n - 1], F1[:, n:n + 1]], axis=1)
    Zb = _sg(sg_c1_blob, F0, F1b)
    s_tol = float(F1[0, n - 1] - F1[0, n]) * 1.01 + 1e-12
    for thr in (0.2, 0.0):
        counts, bad = classify_e2e_disagreements([F0, F1a], [F0, F1b], Za, Zb, thr, s_tol, 1e-6, k=n)
        assert set(counts) == set(E2E_CLASSES)
        # matches through the swapped keypoint are explained by the cut; nothing else may be unexplained
        # beyond decisions whose Z the swap itself moved (z_tol is tight here, so those show up as
        # unexplained and are counted, not hidden)
        assert counts["absent_near_cut"] >= (1 if thr == 0.0 else 0)
        assert counts["unexplained"] == len(bad)
    # with the score margin below the gap, the same swap is unexplained
    counts, bad = classify_e2e_disagreements([F0, F1a], [F0, F1b], Za, Zb, 0.0, 0.0, 1e-6, k=n)
    assert counts["absent_near_cut"] == 0 and counts["unexplained"] >= 1
