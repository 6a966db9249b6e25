"""ORACLE (test infrastructure only): a plain-Python restatement of the reference's line DETECTOR,
LineDetector::LineExtractor's first two steps (src/line_processor.cc:455-470):

    cv::resize(image, smaller_image, cv::Size(), 0.5, 0.5, cv::INTER_LINEAR);
    fld->detect(smaller_image, cv_lines);     // FastLineDetector(length_threshold, distance_threshold,
                                               //   canny_th1, canny_th2, canny_aperture_size, false)

with the configs' parameters (configs/configs_euroc.yaml:31-35: 10, 1.414213562, 200, 250, 3).  It is
the checker of librspl's rspl_lines_detect (csrc/line_kernels.hip resize + Sobel + Canny
classification on the GPU, csrc/lines.cpp hysteresis + chaining + segment fitting on the host),
never called by it.

OpenCV (core imgproc + contrib ximgproc) is a third-party dependency that is NOT vendored in the
reference and not installed here (version unpinned): what follows restates its published
algorithms -- cv::resize's fixed-point bilinear kernel at scale 1/2 (11-bit coefficients), cv::Canny
(3x3 Sobel with replicated borders, L1 magnitude, the TG22 / TG67 fixed-point direction sectors of
the non-maximum suppression with its strict / non-strict neighbour tests, 8-connected hysteresis),
and FastLineDetector (Lee, Lee, Kim, Kweon, Yang, "Outdoor place recognition in urban environments
using straight lines", ICRA 2014): edge pixels chained from raster-order seeds by the most
direction-consistent 8-neighbour, each chain cut into straight runs (a run starts where the
threshold_length+1 points from i lie within distance_threshold of the line through its ends, then
grows while new points stay within the threshold of the least-squares line -- refitted once before
a point is rejected), segment endpoints = the run's first and last points projected on its
least-squares line (cv::fitLine DIST_L2: centroid + principal direction atan2(2 sxy, sxx - syy) / 2),
short and border-hugging segments dropped, and each segment oriented by the mean intensity
difference across it (brighter side on the left).  The corner-zeroing of the Canny image that
OpenCV's implementation performs (top-left 6x6 and bottom-right 5x5 pixels) is kept.  Parity with
the reference is UNPINNED: OpenCV is absent and the reference holds no line vectors; the product
is checked against this file bit-exactly on synthetic images.
"""
from __future__ import annotations

import math
from typing import List, Tuple

import numpy as np

TG22 = int(0.4142135623730950488016887242097 * (1 << 15) + 0.5)  # canny.cpp fixed-point tan(22.5 deg)


def resize_half(img: np.ndarray) -> np.ndarray:
    """cv::resize(0.5, 0.5, INTER_LINEAR) of an even-sized u8 image: source x = 2 dx + 0.5, so both
    taps weigh 1024 / 2048 in each direction and the fixed-point result is (a + b + c + d + 2) >> 2"""
    H, W = img.shape
    assert H % 2 == 0 and W % 2 == 0, "even image sizes only"
    a = img.astype(np.int32)
    s = a[0::2, 0::2] + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2]
    return ((s + 2) >> 2).astype(np.uint8)


def sobel3(img: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """cv::Sobel(ksize 3, CV_16S) of a u8 image with BORDER_REPLICATE: dx, dy as int32"""
    p = np.pad(img.astype(np.int32), 1, mode="edge")
    H, W = img.shape
    sl = lambda dy, dx: p[1 + dy:1 + dy + H, 1 + dx:1 + dx + W]
    dx = (sl(-1, 1) - sl(-1, -1)) + 2 * (sl(0, 1) - sl(0, -1)) + (sl(1, 1) - sl(1, -1))
    dy = (sl(1, -1) - sl(-1, -1)) + 2 * (sl(1, 0) - sl(-1, 0)) + (sl(1, 1) - sl(-1, 1))
    return dx, dy


def canny_classes(img: np.ndarray, th1: float, th2: float) -> np.ndarray:
    """cv::Canny's per-pixel classification before the hysteresis (L1 gradient, aperture 3):
    2 = strong edge (passes the non-maximum suppression and m > high), 0 = candidate (passes it,
    m > low), 1 = no edge.  Magnitudes outside the image are 0."""
    low, high = (th1, th2) if th1 <= th2 else (th2, th1)
    low, high = math.floor(low), math.floor(high)
    dx, dy = sobel3(img)
    m = np.abs(dx) + np.abs(dy)
    H, W = img.shape
    mp = np.zeros((H + 2, W + 2), np.int64)
    mp[1:-1, 1:-1] = m
    at = lambda r, c: mp[1 + r:1 + r + H, 1 + c:1 + c + W]  # neighbour magnitude at offset (r, c)
    x = np.abs(dx).astype(np.int64)
    y = np.abs(dy).astype(np.int64) << 15
    tg22x = x * TG22
    tg67x = tg22x + (x << 16)
    m64 = m.astype(np.int64)
    horiz = y < tg22x
    vert = ~horiz & (y > tg67x)
    diag = ~horiz & ~vert
    s_neg = (dx ^ dy) < 0  # s = -1
    ok_h = (m64 > at(0, -1)) & (m64 >= at(0, 1))
    ok_v = (m64 > at(-1, 0)) & (m64 >= at(1, 0))
    # s = +1: previous row at j - 1, next row at j + 1; s = -1: previous row j + 1, next row j - 1
    ok_dp = (m64 > at(-1, -1)) & (m64 > at(1, 1))
    ok_dn = (m64 > at(-1, 1)) & (m64 > at(1, -1))
    ok_d = np.where(s_neg, ok_dn, ok_dp)
    nms = np.where(horiz, ok_h, np.where(vert, ok_v, ok_d)) & (m64 > low)
    cls = np.ones((H, W), np.uint8)
    cls[nms] = 0
    cls[nms & (m64 > high)] = 2
    return cls


def hysteresis(cls: np.ndarray) -> np.ndarray:
    """8-connected hysteresis from the strong pixels through the candidates -> edges (u8 0 / 255)"""
    H, W = cls.shape
    edge = cls == 2
    cand = cls == 0
    stack = list(zip(*np.nonzero(edge)))
    while stack:
        r, c = stack.pop()
        for dr in (-1, 0, 1):
            for dc in (-1, 0, 1):
                rr, cc = r + dr, c + dc
                if 0 <= rr < H and 0 <= cc < W and cand[rr, cc]:
                    cand[rr, cc] = False
                    edge[rr, cc] = True
                    stack.append((rr, cc))
    return np.where(edge, 255, 0).astype(np.uint8)


def canny(img: np.ndarray, th1: float, th2: float) -> np.ndarray:
    return hysteresis(canny_classes(img, th1, th2))


# FastLineDetector -----------------------------------------------------------------------------
_NB = ((1, 1), (1, 0), (1, -1), (0, -1), (-1, -1), (-1, 0), (-1, 1), (0, 1))  # (dr, dc), index order


def _chain_step(img: np.ndarray, pt: Tuple[int, int], direction: int, step: int):
    """getPointChain: the next pixel of a chain (or None); step 0 takes the first neighbour in index
    order, later steps the most direction-consistent one (ties to the later index), if within 2"""
    H, W = img.shape
    x, y = pt
    best, best_pt, best_dir = 7.0, None, 0
    for i, (dr, dc) in enumerate(_NB):
        ci, ri = x + dc, y + dr
        if ri < 0 or ri == H or ci < 0 or ci == W or img[ri, ci] == 0:
            continue
        d = i - 8 if i > 4 else i
        if step == 0:
            return (ci, ri), d
        diff = abs(float(d) - direction)
        diff = 8.0 - diff if diff > 4.0 else diff
        if diff <= best:
            best, best_pt, best_dir = diff, (ci, ri), d
    if best < 2.0:
        return best_pt, best_dir
    return None


def _line_through(p, q):
    """homogeneous line through two points, normalised so that |(a, b)| = 1"""
    a = p[1] * 1.0 - q[1] * 1.0
    b = q[0] * 1.0 - p[0] * 1.0
    c = p[0] * 1.0 * q[1] - p[1] * 1.0 * q[0]
    n = math.sqrt(a * a + b * b)
    return a / n, b / n, c / n


def _fit_line(pts):
    """cv::fitLine(DIST_L2) of integer points -> the homogeneous line (unit normal) through the
    centroid along the principal direction"""
    n = len(pts)
    sx = sy = sxx = syy = sxy = 0.0
    for x, y in pts:
        sx += x
        sy += y
        sxx += x * x
        syy += y * y
        sxy += x * y
    cx, cy = sx / n, sy / n
    dxx, dyy, dxy = sxx / n - cx * cx, syy / n - cy * cy, sxy / n - cx * cy
    t = math.atan2(2.0 * dxy, dxx - dyy) / 2.0
    vx, vy = math.cos(t), math.sin(t)
    return _line_through((cx, cy), (cx + vx, cy + vy))


def _dist(l, p) -> float:
    return abs(l[0] * p[0] + l[1] * p[1] + l[2])


def _project(l, p):
    d = l[0] * p[0] + l[1] * p[1] + l[2]
    return p[0] - d * l[0], p[1] - d * l[1]


def extract_segments(points: List[Tuple[int, int]], length_thr: int, dist_thr: float) -> List[Tuple[float, ...]]:
    segs = []
    total = len(points)
    i = 0
    while i + length_thr < total:
        ps, pe = points[i], points[i + length_thr]
        l = _line_through(ps, pe)
        if any(_dist(l, points[i + j]) > dist_thr for j in range(1, length_thr)):
            i += 1
            continue
        run = points[i:i + length_thr + 1]
        l = _fit_line(run)
        j = i + length_thr + 1
        while j < total:
            pt = points[j]
            if _dist(l, pt) > dist_thr:
                l = _fit_line(run)
                if _dist(l, pt) > dist_thr:
                    break
            run.append(pt)
            j += 1
        l = _fit_line(run)
        x1, y1 = _project(l, run[0])
        x2, y2 = _project(l, run[-1])
        segs.append((x1, y1, x2, y2))
        i = j  # the rejected point (or the end) starts the next search
    return segs


def _orient(img: np.ndarray, seg):
    """the segment's direction with the brighter side on its left: the intensity difference at
    +-1.5 px along the normal, summed over one sample per pixel of length"""
    H, W = img.shape
    x1, y1, x2, y2 = seg
    dx, dy = x2 - x1, y2 - y1
    L = math.sqrt(dx * dx + dy * dy)
    nx, ny = -dy / L, dx / L
    n = max(1, int(L))
    acc = 0
    for k in range(n):
        t = (k + 0.5) / n
        px, py = x1 + t * dx, y1 + t * dy
        lx, ly = int(math.floor(px + 1.5 * nx + 0.5)), int(math.floor(py + 1.5 * ny + 0.5))
        rx, ry = int(math.floor(px - 1.5 * nx + 0.5)), int(math.floor(py - 1.5 * ny + 0.5))
        if 0 <= lx < W and 0 <= ly < H and 0 <= rx < W and 0 <= ry < H:
            acc += int(img[ly, lx]) - int(img[ry, rx])
    return (x2, y2, x1, y1) if acc < 0 else seg


def fld_detect(img: np.ndarray, length_threshold: int = 10, distance_threshold: float = 1.414213562,
               canny_th1: float = 200.0, canny_th2: float = 250.0) -> np.ndarray:
    """FastLineDetector::detect on a u8 image (do_merge false): segments [n][4] float32 (x1 y1 x2 y2)"""
    H, W = img.shape
    e = canny(img, canny_th1, canny_th2).copy()
    e[0:6, 0:6] = 0
    e[H - 5:H, W - 5:W] = 0
    out = []
    for r in range(H):
        for c in range(W):
            if e[r, c] == 0:
                continue
            pt = (c, r)
            pts = [pt]
            e[r, c] = 0
            direction, step = 0, 0
            while True:
                nxt = _chain_step(e, pt, direction, step)
                if nxt is None:
                    break
                pt, direction = nxt
                pts.append(pt)
                step += 1
                e[pt[1], pt[0]] = 0
            if len(pts) < length_threshold + 1:
                continue
            for seg in extract_segments(pts, length_threshold, distance_threshold):
                x1, y1, x2, y2 = (float(np.float32(v)) for v in seg)  # SEGMENT holds floats
                ddx, ddy = np.float32(x1) - np.float32(x2), np.float32(y1) - np.float32(y2)
                length = np.sqrt(np.float32(ddx * ddx + ddy * ddy))  # float length (float sqrt)
                if length < length_threshold:
                    continue
                if ((x1 <= 5.0 and x2 <= 5.0) or (y1 <= 5.0 and y2 <= 5.0) or
                        (x1 >= W - 5.0 and x2 >= W - 5.0) or (y1 >= H - 5.0 and y2 >= H - 5.0)):
                    continue
                out.append(_orient(img, (x1, y1, x2, y2)))
    return np.array(out, np.float32).reshape(-1, 4)


def line_detect(image: np.ndarray, **kw) -> np.ndarray:
    """LineExtractor's detector step: FLD segments of the half-size image (as fld->detect returns
    them; lines_ref.line_extractor applies the x2 scale and the merges)"""
    return fld_detect(resize_half(image), **kw)
