"""ORACLE (test infrastructure only) -- numpy restatement of the reference's
host-side C++ around the networks.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module; the product path never does.

Each function cites the reference lines it restates (paths relative to the
reference root, llliuqingyu/RSPL-SLAM).  Tie-break documented where the
reference is unspecified (std::sort is not stable: SURVEY.md F7).
"""
from __future__ import annotations

import numpy as np

FLT_MAX = np.float32(3.4028234663852886e38)


def image_to_input(img_u8: np.ndarray) -> np.ndarray:
    """src/super_point.cpp:146-150: float(u8) / 255.0 (double division, stored as float)."""
    return (img_u8.astype(np.float64) / 255.0).astype(np.float32)


def sp_postprocess(scores: np.ndarray, desc: np.ndarray, threshold: float = 0.004,
                   border: int = 4, k: int = 400) -> np.ndarray:
    """SuperPoint::process_output (src/super_point.cpp:285-319) -> 259 x n float64 (column per keypoint).

    scores: [H, W] float32 NMS'd score map; desc: [256, H/8, W/8] float32 (L2-normalised).
    Returns F with F[:, i] = (score, x, y, desc[256]) exactly as the Eigen matrix columns.
    """
    H, W = scores.shape
    flat = scores.reshape(-1)
    # find_high_score_index (:224-235): row-major scan, float > double threshold
    idx = np.nonzero(flat.astype(np.float64) > threshold)[0]
    rows, cols = idx // W, idx % W
    sc = flat[idx]
    # remove_borders (:238-253): keep border <= r < H-border, border <= c < W-border; swap to (x, y)
    keep = (rows >= border) & (rows < H - border) & (cols >= border) & (cols < W - border)
    rows, cols, sc, idx = rows[keep], cols[keep], sc[keep], idx[keep]
    # top_k_keypoints (:262-274): only if k < n and k != -1; sort by score desc.
    # Tie-break (reference unspecified): flat index ascending.
    n = sc.size
    if k != -1 and k < n:
        order = np.lexsort((idx, -sc.astype(np.float64)))[:k]
        rows, cols, sc = rows[order], cols[order], sc[order]
    desc_out = sample_descriptors(cols, rows, desc)
    F = np.empty((259, sc.size), dtype=np.float64)
    F[0] = sc.astype(np.float64)
    F[1] = cols.astype(np.float64)
    F[2] = rows.astype(np.float64)
    F[3:] = desc_out.T
    return F


def sample_descriptors(xs: np.ndarray, ys: np.ndarray, desc: np.ndarray, s: int = 8) -> np.ndarray:
    """normalize_keypoints + grid_sample + normalize_descriptors (src/super_point.cpp:206-283).

    Bilinear with align_corners=True semantics, computed in float64 over the float32 map.
    Returns [n, 256] float64.
    """
    dim, h, w = desc.shape
    x = xs.astype(np.float64)
    y = ys.astype(np.float64)
    # normalize_keypoints (:276-287): s/2 is integer division
    gx = (x - s // 2 + 0.5) / (w * s - s // 2 - 0.5) * 2 - 1
    gy = (y - s // 2 + 0.5) / (h * s - s // 2 - 0.5) * 2 - 1
    # grid_sample (:294-332)
    ix = ((gx + 1) / 2) * (w - 1)
    iy = ((gy + 1) / 2) * (h - 1)

    def clip(v, m):
        return np.minimum(np.maximum(v, 0), m - 1)

    ix_nw = clip(np.floor(ix).astype(np.int64), w)
    iy_nw = clip(np.floor(iy).astype(np.int64), h)
    ix_ne, iy_ne = clip(ix_nw + 1, w), clip(iy_nw, h)
    ix_sw, iy_sw = clip(ix_nw, w), clip(iy_nw + 1, h)
    ix_se, iy_se = clip(ix_nw + 1, w), clip(iy_nw + 1, h)
    nw = (ix_se - ix) * (iy_se - iy)
    ne = (ix - ix_sw) * (iy_sw - iy)
    sw = (ix_ne - ix) * (iy - iy_ne)
    se = (ix - ix_nw) * (iy - iy_nw)
    d = desc.astype(np.float64)
    out = (d[:, iy_nw, ix_nw] * nw + d[:, iy_ne, ix_ne] * ne) + d[:, iy_sw, ix_sw] * sw
    out = out + d[:, iy_se, ix_se] * se           # [256, n]
    out = out.T.copy()
    # normalize_descriptors (:339-345): sequential double inner product, then *= 1/norm
    if out.shape[0]:
        ss = np.cumsum(out * out, axis=1)[:, -1]
        inv = 1.0 / np.sqrt(ss)
        out = inv[:, None] * out
    return out


def normalize_keypoints(F: np.ndarray, width: int, height: int) -> np.ndarray:
    """PointMatching::NormalizeKeypoints (src/point_matching.cc:50-62); width/2 is integer division."""
    G = F.copy()
    scale = max(width, height) * 0.7
    G[1] = (F[1] - width // 2) / scale
    G[2] = (F[2] - height // 2) / scale
    return G


def sg_inputs(F: np.ndarray):
    """SuperGlue::process_input (src/super_glue.cpp:199-246): float32 kpts [N,2], scores [N], desc [256,N]."""
    kpts = F[1:3].T.astype(np.float32)
    scores = F[0].astype(np.float32)
    desc = F[3:].astype(np.float32)
    return kpts, scores, desc


def decode(Z: np.ndarray, threshold: float = 0.2):
    """decode (src/super_glue.cpp:258-367) on the (N+1) x (M+1) float32 log-assignment.

    Returns indices0 [N] int32, indices1 [M] int32, mscores0 [N] float64, mscores1 [M] float64.
    """
    Z = np.asarray(Z, dtype=np.float32)
    h, w = Z.shape
    S = Z[:h - 1, :w - 1]
    n, m = S.shape
    # max_matrix (:258-286): strict '<' from -FLT_MAX -> first maximum wins
    if m:
        max0 = np.argmax(S, axis=1).astype(np.int32)
        val0 = np.maximum(S.max(axis=1), -FLT_MAX)
    else:
        max0 = np.zeros(n, np.int32)
        val0 = np.full(n, -FLT_MAX, np.float32)
    if n:
        max1 = np.argmax(S, axis=0).astype(np.int32)
    else:
        max1 = np.zeros(m, np.int32)
    # equal_gather (:288-296)
    mutual0 = max1[max0] == np.arange(n) if (n and m) else np.zeros(n, bool)
    mutual1 = max0[max1] == np.arange(m) if (n and m) else np.zeros(m, bool)
    # where_exp (:298-306): std::exp on float -> float, stored as double
    ms0 = np.where(mutual0, np.exp(val0.astype(np.float32)).astype(np.float64), 0.0)
    # where_gather (:308-317)
    ms1 = np.where(mutual1, ms0[max1] if n else 0.0, 0.0)
    # and_threshold / and_gather (:319-337)
    valid0 = mutual0 & (ms0 > threshold)
    valid1 = mutual1 & (valid0[max1] if n else False)
    idx0 = np.where(valid0, max0, -1).astype(np.int32)
    idx1 = np.where(valid1, max1, -1).astype(np.int32)
    return idx0, idx1, ms0, ms1


def match_points(idx0, idx1, ms0, ms1):
    """PointMatching::MatchingPoints mutual re-check + DMatch (src/point_matching.cc:24-31).

    Returns int32 [K,2] (query, train) and float32 [K] distances (cv::DMatch stores float).
    """
    q, t, d = [], [], []
    m = len(idx1)
    for i in range(len(idx0)):
        j = int(idx0[i])
        if j < m and j >= 0 and int(idx1[j]) == i:
            q.append(i)
            t.append(j)
            d.append(np.float32(1.0 - (ms0[i] + ms1[j]) / 2.0))
    return np.array(list(zip(q, t)), dtype=np.int32).reshape(-1, 2), np.array(d, dtype=np.float32)
