"""Dataset I/O and trajectory evaluation around the map.

* ``Dataset``: src/dataset.cc:8-50 -- stereo image lists from ``<root>/cam0/data`` and
  ``<root>/cam1/data`` (sorted file names), timestamps parsed from EuRoC-style names
  (``atof(name[0:10]) + atof(name[10:28]) / 1e9``, :17-27; the current time when names are shorter
  than 18 characters), images read as 8-bit grayscale (cv::imread(path, 0), :45-46; here PIL, which
  decodes EuRoC's 8-bit grayscale PNGs to the same bytes).
* ``write_tum`` / ``read_tum``: the TUM lines of Map::SaveKeyframeTrajectory (src/map.cc:1007-1024,
  ``t tx ty tz qx qy qz qw``, std::fixed, setprecision(9)); the native writer is
  ``mapping.Map.SaveKeyframeTrajectory`` (rspl_map_save_trajectory), this one serves trajectories
  held in Python.
* ``ape``: the evaluation run_batch.py:48 runs, ``evo_ape tum gt est -a`` -- timestamp
  association (max 0.01 s), SE(3) Umeyama alignment of the estimate to the reference (no scale),
  statistics of the translation error.  Restated from evo's published algorithm
  (evo.core.sync.matching_time_indices, evo.core.geometry.umeyama_alignment); evo itself is not
  installed here.
"""
from __future__ import annotations

import os
import re
import time
from typing import List, Tuple

import numpy as np


def _atof(s: str) -> float:
    """C atof: the longest leading decimal number (0.0 when there is none)."""
    m = re.match(r"\s*[+-]?(\d+\.?\d*([eE][+-]?\d+)?|\.\d+([eE][+-]?\d+)?)", s)
    return float(m.group(0)) if m else 0.0


class Dataset:
    """Dataset (include/dataset.h, src/dataset.cc:8-50)."""

    def __init__(self, dataroot: str):
        if not os.path.exists(dataroot):
            raise FileNotFoundError(f"dataroot : {dataroot} doesn't exist")
        ld = os.path.join(dataroot, "cam0/data")
        rd = os.path.join(dataroot, "cam1/data")
        names = [n for n in (os.listdir(ld) if os.path.isdir(ld) else []) if n not in (".", "..")]
        self.left: List[str] = []
        self.right: List[str] = []
        self.timestamps: List[float] = []
        if not names:
            return
        names.sort()
        use_current_time = len(names[0]) < 18
        for n in names:
            self.left.append(os.path.join(ld, n))
            self.right.append(os.path.join(rd, n))
            if not use_current_time:
                self.timestamps.append(_atof(n[0:10]) + _atof(n[10:28]) / 1e9)

    def GetDatasetLength(self) -> int:
        return len(self.left)

    def GetData(self, idx: int):
        """-> dict(index, image_left, image_right (u8 [H, W]), time) or None."""
        if idx >= len(self.left) or not os.path.isfile(self.left[idx]) or not os.path.isfile(self.right[idx]):
            return None
        from PIL import Image
        load = lambda p: np.asarray(Image.open(p).convert("L"), dtype=np.uint8)
        t = time.time() if not self.timestamps else self.timestamps[idx]
        return dict(index=idx, image_left=load(self.left[idx]), image_right=load(self.right[idx]), time=t)


def quat_from_R(R) -> np.ndarray:
    """Eigen Quaterniond(Matrix3d) -> (x, y, z, w) (not normalised, as the reference prints it)."""
    t = R[0, 0] + R[1, 1] + R[2, 2]
    q = np.zeros(4)
    if t > 0:
        t = np.sqrt(t + 1.0)
        q[3] = 0.5 * t
        t = 0.5 / t
        q[0], q[1], q[2] = (R[2, 1] - R[1, 2]) * t, (R[0, 2] - R[2, 0]) * t, (R[1, 0] - R[0, 1]) * t
    else:
        i = 0
        if R[1, 1] > R[0, 0]:
            i = 1
        if R[2, 2] > R[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = np.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0)
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (R[k, j] - R[j, k]) * t
        q[j] = (R[j, i] + R[i, j]) * t
        q[k] = (R[k, i] + R[i, k]) * t
    return q


def tum_lines(timestamps, Twc) -> List[str]:
    out = []
    for ts, T in zip(timestamps, Twc):
        T = np.asarray(T)
        q = quat_from_R(T[:3, :3])
        out.append("%.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f" % (ts, T[0, 3], T[1, 3], T[2, 3], q[0], q[1], q[2], q[3]))
    return out


def write_tum(path: str, timestamps, Twc):
    with open(path, "w") as f:
        for line in tum_lines(timestamps, Twc):
            f.write(line + "\n")


def read_tum(path: str) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """-> (timestamps [n], positions [n][3], quaternions [n][4] (x, y, z, w)); '#' lines skipped."""
    rows = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            rows.append([float(v) for v in line.replace(",", " ").split()[:8]])
    a = np.array(rows, np.float64).reshape(-1, 8)
    return a[:, 0], a[:, 1:4], a[:, 4:8]


def tum_line_strings(ts, p, q) -> List[str]:
    return ["%.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f" % (t, *x, *y) for t, x, y in zip(ts, p, q)]


def matching_time_indices(stamps_1, stamps_2, max_diff: float = 0.01, offset_2: float = 0.0):
    """evo.core.sync.matching_time_indices: nearest stamp of 2 for every stamp of 1 within max_diff."""
    s2 = np.asarray(stamps_2, np.float64) + offset_2
    i1, i2 = [], []
    for a, s in enumerate(np.asarray(stamps_1, np.float64)):
        d = np.abs(s2 - s)
        b = int(np.argmin(d))
        if d[b] <= max_diff:
            i1.append(a)
            i2.append(b)
    return i1, i2


def umeyama(x: np.ndarray, y: np.ndarray, with_scale: bool = False):
    """evo.core.geometry.umeyama_alignment: (r, t, c) minimising || y - (c r x + t) || for m x n
    point sets x, y (columns are points)."""
    m, n = x.shape
    mx, my = x.mean(axis=1), y.mean(axis=1)
    sigma_x = 1.0 / n * (np.linalg.norm(x - mx[:, None]) ** 2)
    outer = np.zeros((m, m))
    for i in range(n):
        outer += np.outer(y[:, i] - my, x[:, i] - mx)
    cov = outer / n
    u, d, v = np.linalg.svd(cov)
    s = np.eye(m)
    if np.linalg.det(u) * np.linalg.det(v) < 0.0:
        s[m - 1, m - 1] = -1
    r = u @ s @ v
    c = 1 / sigma_x * np.trace(np.diag(d) @ s) if with_scale else 1.0
    t = my - c * r @ mx
    return r, t, c


def ape(ref_ts, ref_p, est_ts, est_p, align: bool = True, max_diff: float = 0.01) -> dict:
    """evo_ape tum ref est [-a]: absolute translation error statistics after association (and SE(3)
    alignment of the estimate to the reference)."""
    ref_ts, est_ts = np.asarray(ref_ts), np.asarray(est_ts)
    ref_p, est_p = np.asarray(ref_p, np.float64), np.asarray(est_p, np.float64)
    # evo associates the shorter trajectory into the longer one
    if len(est_ts) > len(ref_ts):
        i_ref, i_est = matching_time_indices(ref_ts, est_ts, max_diff)
    else:
        i_est, i_ref = matching_time_indices(est_ts, ref_ts, max_diff)
    if len(i_ref) < 3:
        raise ValueError("ape: fewer than 3 associated poses")
    P, Q = ref_p[i_ref], est_p[i_est]
    if align:
        r, t, _ = umeyama(Q.T, P.T, False)
        Q = (r @ Q.T).T + t
    e = np.linalg.norm(P - Q, axis=1)
    return dict(rmse=float(np.sqrt(np.mean(e ** 2))), mean=float(e.mean()), median=float(np.median(e)),
                std=float(e.std()), min=float(e.min()), max=float(e.max()), sse=float(np.sum(e ** 2)),
                n=int(len(e)))
