"""ORACLE (test infrastructure only): a plain-Python restatement of the reference's line front end
after the detector -- the LineDetector merge passes, the point-to-line assignment and the
shared-point line matching -- used to check librspl's csrc/lines.cpp and csrc/line_kernels.hip
(the product), never called by them.

Restated from (file:line of /root/reference):
  src/line_processor.cc:11-39    FilterShortLines (float and double overloads)
  src/line_processor.cc:41-50    PointLineDistance (float, std::pow promotes to double)
  src/line_processor.cc:92-96    AngleDiff (case 2 in double, stored as float)
  src/line_processor.cc:98-161   MergeTwoLines (float endpoints, double centroid / angle; atan of a
                                 float quotient is the float overload, atanf)
  src/line_processor.cc:163-216  AssignPointsToLines (double, the distance stored through a float)
  src/line_processor.cc:221-283  MatchLines (shared matched points, first-max row / column argmax,
                                 score = v^2 / min(|points on line|) >= 0.8)
  src/line_processor.cc:460-490  LineDetector::LineExtractor after fld->detect: x2 scale, merge
                                 (0.05, 5, 15), filter 30, merge (0.03, 3, 50), filter 60
  src/line_processor.cc:492-665  LineDetector::MergeLines (angle-sorted neighbour search, BFS
                                 clusters, length-ordered sub-clusters, pairwise merge)
  src/frame.cc:150-203           Frame::AddRightFeatures (disparity filter of the stereo matches,
                                 right-line association; line_matches[i] > 0 quirk kept)
Float semantics follow the reference's types exactly (numpy float32 scalars for float, Python
floats for double; atanf through the C library, as the reference's std::atan(float)).  Orders
the reference leaves to std::sort (equal angles, equal lengths) are taken stable here; the tests
use inputs without such ties.  Parity of this file with the reference C++ is unpinned: the
reference's line code needs OpenCV (contrib) and Eigen, absent here, and its tests hold no line
vectors.  The FLD detector and the RCF edge network themselves are not restated (no source for
cv::ximgproc in the image, no RCF weights in the reference).
"""
from __future__ import annotations

import ctypes
import math
from typing import Dict, List, Sequence

import numpy as np

f32 = np.float32
_libm = ctypes.CDLL("libm.so.6")
_libm.atanf.restype = ctypes.c_float
_libm.atanf.argtypes = [ctypes.c_float]


def atanf(x) -> np.float32:
    return f32(_libm.atanf(ctypes.c_float(float(x))))


def filter_short_lines(lines: List[np.ndarray], length_thr: float) -> List[np.ndarray]:
    """:11-39 -- squared length (in the lines' own precision) > thr^2 (float)."""
    thr = f32(length_thr)
    thr2 = f32(thr * thr)
    out = []
    for ln in lines:
        dx = ln[2] - ln[0]
        dy = ln[3] - ln[1]
        if dx * dx + dy * dy > thr2:
            out.append(ln)
    return out


def point_line_distance(line: np.ndarray, pt: np.ndarray) -> np.float32:
    """:41-50 -- float numerator, double denominator (std::pow(float, int) is a double)."""
    x0, y0 = pt[0], pt[1]
    x1, y1, x2, y2 = line[0], line[1], line[2], line[3]
    num = abs(((y2 - y1) * x0 + (x1 - x2) * y0) + ((x2 * y1) - (x1 * y2)))
    den = math.sqrt(float(y2 - y1) ** 2 + float(x1 - x2) ** 2)
    return f32(float(num) / den)


def angle_diff(a1: np.float32, a2: np.float32) -> np.float32:
    """:92-96"""
    c1 = abs(a2 - a1)
    c2 = f32(math.pi + float(min(a1, a2)) - float(max(a1, a2)))
    return min(c1, c2)


def merge_two_lines(l1: np.ndarray, l2: np.ndarray) -> np.ndarray:
    """:98-161"""
    ax, ay, bx, by = l1[0], l1[1], l1[2], l1[3]
    cx, cy, dx, dy = l2[0], l2[1], l2[2], l2[3]
    dlix, dliy, dljx, dljy = bx - ax, by - ay, dx - cx, dy - cy
    li = math.sqrt(float(dlix * dlix) + float(dliy * dliy))
    lj = math.sqrt(float(dljx * dljx) + float(dljy * dljy))
    xg = (li * float(ax + bx) + lj * float(cx + dx)) / (2.0 * (li + lj))
    yg = (li * float(ay + by) + lj * float(cy + dy)) / (2.0 * (li + lj))
    with np.errstate(divide="ignore", invalid="ignore"):
        thi = math.pi / 2.0 if dlix == f32(0) else float(atanf(dliy / dlix))
        thj = math.pi / 2.0 if dljx == f32(0) else float(atanf(dljy / dljx))
    if abs(thi - thj) <= math.pi / 2.0:
        thr = (li * thi + lj * thj) / (li + lj)
    else:
        tmp = thj - math.pi * (thj / abs(thj))
        thr = (li * thi + lj * tmp) / (li + lj)
    s, c = math.sin(thr), math.cos(thr)
    axg = (float(ay) - yg) * s + (float(ax) - xg) * c
    bxg = (float(by) - yg) * s + (float(bx) - xg) * c
    cxg = (float(cy) - yg) * s + (float(cx) - xg) * c
    dxg = (float(dy) - yg) * s + (float(dx) - xg) * c
    d1 = min(axg, min(bxg, min(cxg, dxg)))
    d2 = max(axg, max(bxg, max(cxg, dxg)))
    return np.array([d1 * math.cos(thr) + xg, d1 * math.sin(thr) + yg,
                     d2 * math.cos(thr) + xg, d2 * math.sin(thr) + yg], dtype=f32)


def merge_neighbors(src: List[np.ndarray], angle_threshold: float, distance_threshold: float,
                    endpoint_threshold: float):
    """:495-589 -- the neighbour lists (in the reference's push_back order) and the angles."""
    n = len(src)
    with np.errstate(divide="ignore", invalid="ignore"):  # dx == 0: +-inf -> +-pi/2, as atanf
        angles = [atanf((ln[3] - ln[1]) / (ln[2] - ln[0])) for ln in src]
    order = sorted(range(n), key=lambda i: angles[i])
    ang_thr = f32(angle_threshold)
    dist_thr = f32(distance_threshold)
    ep = f32(endpoint_threshold)
    ep_thr = f32(ep * ep)
    quarter = f32(math.pi / 4.0)
    nbr: List[List[int]] = [[] for _ in range(n)]
    for i in range(n):
        i1 = order[i]
        x11, y11, x12, y12 = src[i1]
        a1 = angles[i1]
        sx = abs(a1) < quarter
        if (sx and x12 < x11) or ((not sx) and y12 < y11):
            x11, x12 = x12, x11
            y11, y12 = y12, y11
        for j in range(i + 1, n):
            i2 = order[j]
            x21, y21, x22, y22 = src[i2]
            if (sx and x22 < x21) or ((not sx) and y22 < y21):
                x21, x22 = x22, x21
                y21, y22 = y22, y21
            da = angle_diff(a1, angles[i2])
            if da > ang_thr:
                if abs(float(a1)) < (math.pi / 2 - float(ang_thr)):
                    break
                continue
            m1 = f32(0.5) * (src[i1][0:2] + src[i1][2:4])
            m2 = f32(0.5) * (src[i2][0:2] + src[i2][2:4])
            d12 = point_line_distance(src[i2], m1)
            d21 = point_line_distance(src[i1], m2)
            if d12 > dist_thr and d21 > dist_thr:
                continue
            if (sx and x12 > x22) or ((not sx) and y12 > y22):
                cx12, cy12, cx21, cy21 = x22, y22, x11, y11
            else:
                cx12, cy12, cx21, cy21 = x12, y12, x21, y21
            merge = (sx and cx12 >= cx21) or ((not sx) and cy12 >= cy21)
            if not merge:
                dep = (cx21 - cx12) * (cx21 - cx12) + (cy21 - cy12) * (cy21 - cy12)
                merge = dep < ep_thr
            if merge:
                nbr[i1].append(i2)
                nbr[i2].append(i1)
    return nbr, angles


def merge_lines(src: List[np.ndarray], angle_threshold: float, distance_threshold: float,
                endpoint_threshold: float) -> List[np.ndarray]:
    """:492-665"""
    n = len(src)
    if n == 0:
        return []
    nbr, _ = merge_neighbors(src, angle_threshold, distance_threshold, endpoint_threshold)
    length = [np.sqrt((ln[2] - ln[0]) * (ln[2] - ln[0]) + (ln[3] - ln[1]) * (ln[3] - ln[1])) for ln in src]
    codes = [-1] * n
    clusters: List[List[int]] = []
    for i in range(n):
        if codes[i] >= 0:
            continue
        code = len(clusters)
        codes[i] = code
        todo = list(nbr[i])
        cl = [i]
        while todo:
            tmp = set()
            for j in todo:
                if codes[j] < 0:
                    codes[j] = code
                    cl.append(j)
                for k in nbr[j]:
                    if codes[k] < 0:
                        tmp.add(k)
            todo = sorted(tmp)
        clusters.append(cl)
    subs: List[List[int]] = []
    for cl in clusters:
        if len(cl) <= 2:
            subs.append(cl)
            continue
        cl = sorted(cl, key=lambda i: -float(length[i]))
        loc = {l: p for p, l in enumerate(cl)}
        done = [False] * len(cl)
        for j in range(len(cl)):
            if done[j]:
                continue
            li = cl[j]
            sub = [li]
            for k in nbr[li]:
                done[loc[k]] = True
                sub.append(k)
            subs.append(sub)
    out = []
    for sub in subs:
        ln = src[sub[0]].copy()
        for i in sub[1:]:
            ln = merge_two_lines(ln, src[i])
        out.append(ln)
    return out


def line_extractor(cv_lines: np.ndarray, do_merge: bool = True) -> np.ndarray:
    """:460-490 after fld->detect on the half-size image: segments [n][4] float -> lines [m][4]
    double (x2 scale, then the two merge / filter passes)."""
    src = [np.asarray(l, dtype=f32) * f32(2) for l in np.asarray(cv_lines, dtype=f32).reshape(-1, 4)]
    if do_merge and src:
        tmp = filter_short_lines(merge_lines(src, 0.05, 5, 15), 30)
        dst = filter_short_lines(merge_lines(tmp, 0.03, 3, 50), 60) if tmp else []
    else:
        dst = src
    return np.array([l.astype(np.float64) for l in dst], dtype=np.float64).reshape(-1, 4)


def assign_points_to_lines(lines: np.ndarray, xy: np.ndarray) -> List[Dict[int, float]]:
    """:163-216 -- lines [n][4] double, keypoints xy [N][2] double (features rows 1, 2)."""
    rel: List[Dict[int, float]] = []
    for (x1, y1, x2, y2) in np.asarray(lines, dtype=np.float64).reshape(-1, 4):
        x1, y1, x2, y2 = float(x1), float(y1), float(x2), float(y2)
        A, B, C = y2 - y1, x1 - x2, x2 * y1 - x1 * y2
        D = math.sqrt(A * A + B * B)
        lo_x, hi_x = (x2, x1) if x1 > x2 else (x1, x2)
        lo_y, hi_y = (y2, y1) if y1 > y2 else (y1, y2)
        pts: Dict[int, float] = {}
        for j, (px, py) in enumerate(np.asarray(xy, dtype=np.float64).reshape(-1, 2)):
            px, py = float(px), float(py)
            if px < lo_x - 3 or px > hi_x + 3 or py < lo_y - 3 or py > hi_y + 3:
                continue
            d = f32(abs(A * px + B * py + C) / D)
            if d > 6:
                continue
            s1 = (x1 - px) ** 2 + (y1 - py) ** 2
            s2 = (x2 - px) ** 2 + (y2 - py) ** 2
            ls = D * D
            if s1 <= 9 or s2 <= 9 or (s1 < ls + s2 and s2 < ls + s1):
                pts[j] = float(d)
        rel.append(pts)
    return rel


def match_lines(pol0: Sequence[Dict[int, float]], pol1: Sequence[Dict[int, float]],
                matches: np.ndarray, n_points0: int, n_points1: int) -> List[int]:
    """:221-283 -- matches [m][2] (queryIdx, trainIdx)."""
    n0, n1 = len(pol0), len(pol1)
    out = [-1] * n0
    if n_points0 == 0 or n_points1 == 0 or n0 == 0 or n1 == 0:
        return out
    a0: List[List[int]] = [[] for _ in range(n_points0)]
    a1: List[List[int]] = [[] for _ in range(n_points1)]
    for i, m in enumerate(pol0):
        for p in m:
            a0[p].append(i)
    for i, m in enumerate(pol1):
        for p in m:
            a1[p].append(i)
    M = np.zeros((n0, n1), dtype=np.int64)
    for q, t in np.asarray(matches, dtype=np.int64).reshape(-1, 2):
        for l0 in a0[q]:
            for l1 in a1[t]:
                M[l0, l1] += 1
    row_loc = M.argmax(axis=1)  # first maximum, as Eigen's maxCoeff(&index)
    for j in range(n1):
        cm = int(M[:, j].argmax())
        v = int(M[cm, j])
        if v < 2 or row_loc[cm] != j:
            continue
        score = f32(v * v) / f32(min(len(pol0[cm]), len(pol1[j])))
        if score < f32(0.8):
            continue
        out[cm] = j
    return out


def stereo_filter(xl: np.ndarray, xr: np.ndarray, yl: np.ndarray, yr: np.ndarray, matches: np.ndarray,
                  min_x_diff: float, max_x_diff: float, max_y_diff: float) -> np.ndarray:
    """frame.cc:157-167 -- the stereo matches kept for triangulation and line matching."""
    keep = []
    for q, t in np.asarray(matches, dtype=np.int64).reshape(-1, 2):
        dx = abs(float(xl[q]) - float(xr[t]))
        dy = abs(float(yl[q]) - float(yr[t]))
        if min_x_diff < dx < max_x_diff and dy <= max_y_diff:
            keep.append((q, t))
    return np.array(keep, dtype=np.int64).reshape(-1, 2)


def right_lines(lines_right: np.ndarray, line_matches: Sequence[int], n_left: int):
    """frame.cc:185-196 -- right line of each left line; valid only for line_matches[i] > 0 (the
    reference's test: a match to right line 0 counts as invalid)."""
    out = np.zeros((n_left, 4))
    valid = np.zeros(n_left, dtype=bool)
    for i in range(n_left):
        if line_matches[i] > 0:
            out[i] = lines_right[line_matches[i]]
            valid[i] = True
    return out, valid
