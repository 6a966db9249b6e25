"""Seeded synthetic inputs shaped like the reference's workloads.

EuRoC / OIVIO images are not available, so benches and tests
use seeded textured images with EuRoC geometry (752x480 u8), synthetic
SuperGlue keypoint sets, and synthetic local-BA problems with ground truth.
Everything here is numpy, deterministic for a given seed.
"""
from __future__ import annotations

import numpy as np

# EuRoC rectified intrinsics: configs/euroc.yaml:7 (bf) and LEFT.P (:32-36)
EUROC_FX = 435.2046959714599
EUROC_FY = 435.2046959714599
EUROC_CX = 367.4517211914062
EUROC_CY = 252.2008514404297
EUROC_BF = 47.90639384423901


def textured_image(h: int, w: int, seed: int, n_blobs: int = 60) -> np.ndarray:
    """Smooth texture + gaussian blobs + pixel noise, u8 [h, w]."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    img = 128 + 40 * np.sin(xx / 7.3) * np.cos(yy / 5.1) + 30 * np.sin((xx + yy) / 13.7)
    for _ in range(n_blobs):
        cx, cy, r = rng.uniform(0, w), rng.uniform(0, h), rng.uniform(3, 25)
        img += rng.uniform(-60, 60) * np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * r * r))
    img += rng.normal(0, 6, size=img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def stereo_pair(h: int, w: int, seed: int, disparity: int = 12):
    """Left/right u8 images: the right view is the left texture shifted by a constant disparity
    plus independent sensor noise (rectified stereo, as after Camera::UndistortImage)."""
    base = textured_image(h, w + disparity, seed).astype(np.float64)
    rng = np.random.default_rng(seed + 1000)
    left = base[:, disparity:]
    right = base[:, :w]
    right = right + rng.normal(0, 2, size=right.shape)
    return left.astype(np.uint8), np.clip(right, 0, 255).astype(np.uint8)


def sg_problem(n0: int, n1: int, n_common: int, seed: int, width: int = 752, height: int = 480):
    """Two 259 x n feature matrices (score, x, y, desc[256]) in IMAGE coordinates (not normalised),
    where n_common keypoints of image 1 are noisy copies of image-0 keypoints.
    Returns (F0, F1, gt) with gt[j] = index in image 0 of image-1 keypoint j or -1."""
    rng = np.random.default_rng(seed)
    k0 = rng.uniform([0, 0], [width, height], size=(n0, 2))
    d0 = rng.normal(size=(256, n0))
    d0 /= np.linalg.norm(d0, axis=0)
    n_common = min(n_common, n0, n1)
    perm = rng.permutation(n0)[:n_common]
    k1 = np.concatenate([k0[perm] + rng.normal(0, 1.0, size=(n_common, 2)),
                         rng.uniform([0, 0], [width, height], size=(n1 - n_common, 2))])
    d1 = np.concatenate([d0[:, perm] + 0.5 * rng.normal(size=(256, n_common)) / 16,
                         rng.normal(size=(256, n1 - n_common))], 1)
    d1 /= np.linalg.norm(d1, axis=0)
    s0 = rng.uniform(size=n0)
    s1 = rng.uniform(size=n1)
    F0 = np.concatenate([s0[None], k0.T, d0], 0)
    F1 = np.concatenate([s1[None], k1.T, d1], 0)
    gt = np.full(n1, -1, np.int64)
    gt[:n_common] = perm
    return np.ascontiguousarray(F0), np.ascontiguousarray(F1), gt


# ----------------------------------------------------------------------------
# Synthetic local-BA problems (Map::LocalMapOptimization shapes, src/map.cc:537-707)
# ----------------------------------------------------------------------------
def _rotvec_to_R(r):
    th = np.linalg.norm(r)
    if th < 1e-12:
        return np.eye(3)
    k = r / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


def R_to_quat_xyzw(R):
    t = np.trace(R)
    if t > 0:
        s = np.sqrt(t + 1.0) * 2
        w, x, y, z = 0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s
    else:
        i = int(np.argmax(np.diag(R)))
        j, k = (i + 1) % 3, (i + 2) % 3
        s = np.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0) * 2
        v = np.zeros(3)
        v[i] = 0.25 * s
        w = (R[k, j] - R[j, k]) / s
        v[j] = (R[j, i] + R[i, j]) / s
        v[k] = (R[k, i] + R[i, k]) / s
        x, y, z = v
    q = np.array([x, y, z, w])
    return q / np.linalg.norm(q) * (1 if w >= 0 else -1)


def quat_xyzw_to_R(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def ba_problem(n_poses: int = 10, n_points: int = 2000, n_lines: int = 50, obs_per_point: int = 6,
               pixel_sigma: float = 0.8, outlier_frac: float = 0.05, seed: int = 0,
               init_noise: float = 1.0, width: int = 752, height: int = 480, n_fixed: int = 1,
               cam=(EUROC_FX, EUROC_FY, EUROC_CX, EUROC_CY, EUROC_BF)):
    """Seeded local-BA problem with ground truth.

    Returns (DenseProblem, gt) where gt = dict(pose_q, pose_p, points, lines).  Points are observed
    by ``obs_per_point`` random poses that see them; observations are stereo when the right-image
    coordinate is valid (Frame::AddRightFeatures-style depth range), else mono; ``outlier_frac``
    of the observations get gross (30-80 px) errors.  The first ``n_fixed`` poses are fixed.
    ``init_noise`` scales the perturbation of the initial estimate (0 = start at ground truth).
    """
    from .ba_types import DenseProblem
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = cam
    # trajectory: forward-moving camera with small yaw/pitch wobble (T_wc)
    Rwc, twc = [], []
    for i in range(n_poses):
        r = np.array([0.02 * np.sin(0.7 * i), 0.05 * np.sin(0.3 * i), 0.01 * i])
        Rwc.append(_rotvec_to_R(r))
        twc.append(np.array([0.15 * i, 0.03 * np.sin(0.5 * i), 0.08 * i]))
    # points in front of the rig
    pts = np.stack([rng.uniform(-4, 4 + 0.15 * n_poses, n_points), rng.uniform(-2.5, 2.5, n_points),
                    rng.uniform(3.0, 14.0, n_points) + 0.08 * n_poses * rng.uniform(0, 1, n_points)], 1)

    def project(i, X):
        Xc = Rwc[i].T @ (X - twc[i])
        if Xc[2] <= 0.1:
            return None
        u = fx * Xc[0] / Xc[2] + cx
        v = fy * Xc[1] / Xc[2] + cy
        if not (0 <= u < width and 0 <= v < height):
            return None
        return np.array([u, v, u - bf / Xc[2]]), Xc[2]

    mono = dict(pose=[], lm=[], obs=[])
    stereo = dict(pose=[], lm=[], obs=[])
    keep = []
    for j in range(n_points):
        vis = [i for i in range(n_poses) if project(i, pts[j]) is not None]
        if len(vis) < 2:
            continue
        sel = rng.permutation(vis)[:obs_per_point]
        jj = len(keep)
        keep.append(j)
        for i in sorted(sel):
            uvr, z = project(i, pts[j])
            noisy = uvr + rng.normal(0, pixel_sigma, 3)
            if rng.uniform() < outlier_frac:
                noisy[:2] += rng.uniform(30, 80, 2) * rng.choice([-1, 1], 2)
            if uvr[2] > 0 and z < 10.0 and rng.uniform() < 0.7:   # stereo (right coordinate valid)
                stereo["pose"].append(i); stereo["lm"].append(jj); stereo["obs"].append(noisy)
            else:
                mono["pose"].append(i); mono["lm"].append(jj); mono["obs"].append(noisy[:2])
    pts = pts[keep]

    # lines: segments in front of the rig; Pluecker (w = p x d, d unit)
    lines_gt, mline, sline = [], dict(pose=[], lm=[], obs=[]), dict(pose=[], lm=[], obs=[])
    for _ in range(n_lines):
        p0 = np.array([rng.uniform(-3, 3 + 0.15 * n_poses), rng.uniform(-2, 2), rng.uniform(4, 10)])
        dvec = rng.normal(size=3)
        dvec /= np.linalg.norm(dvec)
        p1 = p0 + dvec * rng.uniform(0.8, 2.0)
        obs_i = []
        for i in range(n_poses):
            a, b = project(i, p0), project(i, p1)
            if a is None or b is None:
                continue
            obs_i.append((i, a[0], b[0]))
        if len(obs_i) < 2:
            continue
        li = len(lines_gt)
        lines_gt.append(np.concatenate([np.cross(p0, dvec), dvec]))
        for (i, a, b) in obs_i[:obs_per_point]:
            nL = rng.normal(0, pixel_sigma, 4)
            ol = np.array([a[0], a[1], b[0], b[1]]) + nL
            if a[2] > 0 and b[2] > 0 and rng.uniform() < 0.5:
                orr = np.array([a[2], a[1], b[2], b[1]]) + rng.normal(0, pixel_sigma, 4)
                sline["pose"].append(i); sline["lm"].append(li); sline["obs"].append(np.concatenate([ol, orr]))
            else:
                mline["pose"].append(i); mline["lm"].append(li); mline["obs"].append(ol)
    lines_gt = np.array(lines_gt).reshape(-1, 6)

    q_gt = np.array([R_to_quat_xyzw(R) for R in Rwc])
    p_gt = np.array(twc)
    # perturbed initial estimate
    q0, p0s = q_gt.copy(), p_gt.copy()
    for i in range(n_fixed, n_poses):
        dR = _rotvec_to_R(rng.normal(0, 0.005 * init_noise, 3))
        q0[i] = R_to_quat_xyzw(dR @ quat_xyzw_to_R(q_gt[i]))
        p0s[i] = p_gt[i] + rng.normal(0, 0.02 * init_noise, 3)
    pts0 = pts + rng.normal(0, 0.05 * init_noise, pts.shape)
    lines0 = lines_gt.copy()
    for k in range(lines0.shape[0]):
        # move the line by a small rigid perturbation of two points on it, then re-derive (w, d)
        d = lines0[k, 3:]
        w = lines0[k, :3]
        pc = np.cross(d, w)   # closest point to origin (|d| = 1)
        pa = pc + rng.normal(0, 0.03 * init_noise, 3)
        da = d + rng.normal(0, 0.01 * init_noise, 3)
        da /= np.linalg.norm(da)
        lines0[k] = np.concatenate([np.cross(pa, da), da])
    fixed = np.zeros(n_poses, np.uint8)
    fixed[:n_fixed] = 1
    arr = lambda d, od: dict(pose=np.array(d["pose"], np.int32), lm=np.array(d["lm"], np.int32),
                             obs=np.array(d["obs"], np.float64).reshape(-1, od))
    prob = DenseProblem(cameras=np.array([cam], np.float64), pose_q=q0, pose_p=p0s, pose_fixed=fixed,
                        points=pts0, lines=lines0, mono=arr(mono, 2), stereo=arr(stereo, 3),
                        mono_line=arr(mline, 4), stereo_line=arr(sline, 8))
    gt = dict(pose_q=q_gt, pose_p=p_gt, points=pts, lines=lines_gt)
    return prob, gt


def frame_problem(n_points: int = 300, pixel_sigma: float = 0.8, outlier_frac: float = 0.1, seed: int = 0,
                  init_rot: float = 0.01, init_trans: float = 0.05, stereo_frac: float = 0.6,
                  width: int = 752, height: int = 480, cam=(EUROC_FX, EUROC_FY, EUROC_CX, EUROC_CY, EUROC_BF)):
    """Seeded FrameOptimization problem (MapBuilder::FramePoseOptimization shape, map_builder.cc:536-580):
    one camera pose, ``n_points`` fixed map points visible in it, a stereo constraint when the right
    coordinate is valid (``stereo_frac`` of them), else mono; ``outlier_frac`` gross mismatches;
    the initial pose is the ground truth perturbed as a PnP initialisation would be.
    Returns (FrameProblem, gt) with gt = dict(pose_q, pose_p)."""
    from .ba_types import FrameProblem
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = cam
    Rwc = _rotvec_to_R(rng.normal(0, 0.1, 3))
    twc = rng.normal(0, 1.0, 3)
    pts, mono, stereo = [], dict(lm=[], obs=[], out=[]), dict(lm=[], obs=[], out=[])
    while len(pts) < n_points:
        u, v, z = rng.uniform(0, width), rng.uniform(0, height), rng.uniform(1.5, 20.0)
        Xc = np.array([(u - cx) / fx * z, (v - cy) / fy * z, z])
        X = Rwc @ Xc + twc
        j = len(pts)
        pts.append(X)
        obs = np.array([u, v, u - bf / z]) + rng.normal(0, pixel_sigma, 3)
        out = rng.uniform() < outlier_frac
        if out:
            obs[:2] += rng.uniform(20, 80, 2) * rng.choice([-1, 1], 2)
        d = stereo if obs[2] > 0 and rng.uniform() < stereo_frac else mono
        d["lm"].append(j); d["obs"].append(obs if d is stereo else obs[:2]); d["out"].append(out)
    dR = _rotvec_to_R(rng.normal(0, init_rot, 3))
    q0 = R_to_quat_xyzw(dR @ Rwc)
    p0 = twc + rng.normal(0, init_trans, 3)
    arr = lambda d, od: dict(lm=np.array(d["lm"], np.int32), obs=np.array(d["obs"], np.float64).reshape(-1, od))
    prob = FrameProblem(cameras=np.array([cam], np.float64), pose_q=q0, pose_p=p0, points=np.array(pts),
                        mono=arr(mono, 2), stereo=arr(stereo, 3))
    return prob, dict(pose_q=R_to_quat_xyzw(Rwc), pose_p=twc, outlier_mono=np.array(mono["out"], bool),
                      outlier_stereo=np.array(stereo["out"], bool))


def pnp_problem(n_points: int = 300, pixel_sigma: float = 0.8, outlier_frac: float = 0.2, seed: int = 0,
                width: int = 752, height: int = 480, cam=(EUROC_FX, EUROC_FY, EUROC_CX, EUROC_CY)):
    """Seeded SolvePnPWithCV input (g2o_optimization.cc:409-431): map points of the last frame
    matched into the current one, ``outlier_frac`` of them mismatched.  Returns
    (K4 = (fx, fy, cx, cy), points [n, 3], keypoints [n, 2], gt) with gt = dict(Rwc, twc, outlier)."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = cam
    Rwc = _rotvec_to_R(rng.normal(0, 0.2, 3))
    twc = rng.normal(0, 1.0, 3)
    u, v = rng.uniform(0, width, n_points), rng.uniform(0, height, n_points)
    z = rng.uniform(1.5, 20.0, n_points)
    Xc = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], 1)
    X = Xc @ Rwc.T + twc
    kp = np.stack([u, v], 1) + rng.normal(0, pixel_sigma, (n_points, 2))
    out = rng.uniform(size=n_points) < outlier_frac
    kp[out] = np.stack([rng.uniform(0, width, out.sum()), rng.uniform(0, height, out.sum())], 1)
    return np.array(cam, np.float64), X, kp, dict(Rwc=Rwc, twc=twc, outlier=out)


# ----------------------------------------------------------------------------
# Synthetic keyframe sequence for the map-side local BA (Map::InsertKeyframe ->
# Map::LocalMapOptimization, src/map.cc:24-118, :537-808)
# ----------------------------------------------------------------------------
def _Twc(R, t):
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t
    return T


def map_sequence(n_keyframes: int = 30, n_points: int = 6000, n_lines: int = 80, seed: int = 0,
                 pixel_sigma: float = 0.8, outlier_frac: float = 0.03, drift: float = 1.0, step: float = 0.25,
                 points_per_line: int = 4, frames_per_keyframe: int = 5, width: int = 752, height: int = 480,
                 cam=(EUROC_FX, EUROC_FY, EUROC_CX, EUROC_CY, EUROC_BF)):
    """What tracking hands the map, keyframe by keyframe, for a forward-moving stereo rig.

    Returns dict(camera, gt_Twc [n][4][4], timestamps [n], keyframes [n]) where keyframe k is a dict:
      id, timestamp, parent_id, Twc (the tracked pose: ground truth with an accumulated drift),
      keypoints [m][3] (x, y, u_right; u_right < 0 = mono), lines_left / lines_right [l][4],
      lines_right_valid [l], points_on_lines [l] {keypoint: distance},
      new_points [(id, p)] (first seen here; p = ground truth + a depth-scaled triangulation error),
      new_lines [(id, Pluecker (w, d))], point_obs [(point id, keypoint)], line_obs [(line id, line)].
    Landmarks are created Good with a position (the reference triangulates them while inserting the
    keyframe, map.cc:41-60 -- outside this path).  ``outlier_frac`` of the observations carry gross
    30-80 px errors, so the BA flags outliers and the map removes them.  Points sampled on the lines
    are associated with them (points_on_lines), so UppdateMapline finds endpoints.
    """
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = cam
    n = n_keyframes
    gt, tracked, ts = [], [], []
    drift_R, drift_t = np.eye(3), np.zeros(3)
    for k in range(n):
        s = k * step
        R = _rotvec_to_R(np.array([0.03 * np.sin(0.4 * k), 0.08 * np.sin(0.15 * k), 0.02 * np.sin(0.3 * k)]))
        t = np.array([0.6 * np.sin(0.12 * k), 0.05 * np.sin(0.3 * k), s])
        gt.append(_Twc(R, t))
        if k > 0:  # tracking drift: a random walk on the pose
            drift_R = _rotvec_to_R(rng.normal(0, 0.002 * drift, 3)) @ drift_R
            drift_t = drift_t + rng.normal(0, 0.006 * drift, 3)
        tracked.append(_Twc(drift_R @ R, t + drift_t))
        ts.append(1403636579.0 + 0.05 * frames_per_keyframe * k)
    zmax = n * step + 14.0
    pts = np.stack([rng.uniform(-7, 7, n_points), rng.uniform(-3.5, 3.5, n_points), rng.uniform(1.5, zmax, n_points)], 1)
    segs = []
    for _ in range(n_lines):
        p0 = np.array([rng.uniform(-5, 5), rng.uniform(-2.5, 2.5), rng.uniform(3, zmax - 2)])
        dv = rng.normal(size=3)
        dv /= np.linalg.norm(dv)
        segs.append((p0, p0 + dv * rng.uniform(1.0, 2.5)))
    # points on the lines (associated with them in the frames)
    on_line = []
    for li, (a, b) in enumerate(segs):
        for u in rng.uniform(0.05, 0.95, points_per_line):
            on_line.append((li, a + u * (b - a)))
    n_free = len(pts)
    pts = np.concatenate([pts, np.array([p for _, p in on_line]).reshape(-1, 3)], 0)
    line_of_point = {n_free + i: li for i, (li, _) in enumerate(on_line)}

    def project(T, X):
        Xc = T[:3, :3].T @ (X - T[:3, 3])
        if Xc[2] <= 0.3 or Xc[2] > 30.0:
            return None
        u, v = fx * Xc[0] / Xc[2] + cx, fy * Xc[1] / Xc[2] + cy
        if not (2 <= u < width - 2 and 2 <= v < height - 2):
            return None
        return np.array([u, v, u - bf / Xc[2]]), Xc[2]

    created_p, created_l = set(), set()
    kfs = []
    for k in range(n):
        T = gt[k]
        kps, pobs, newp = [], [], []
        kp_of_point = {}
        for j in range(len(pts)):
            pr = project(T, pts[j])
            if pr is None or rng.uniform() < 0.1:   # missed detection / not matched
                continue
            uvr, z = pr
            o = uvr + rng.normal(0, pixel_sigma, 3)
            if rng.uniform() < outlier_frac:
                o[:2] += rng.uniform(30, 80, 2) * rng.choice([-1, 1], 2)
            if not (uvr[2] > 0 and z < 12.0 and rng.uniform() < 0.75):
                o[2] = -1.0                          # no right match: mono
            kp_of_point[j] = len(kps)
            kps.append(o)
            if j not in created_p:
                created_p.add(j)
                err = rng.normal(0, 0.01 + 0.004 * z, 3)
                newp.append((j, pts[j] + err))
            pobs.append((j, kp_of_point[j]))
        ll, lr, lv, pol, lobs, newl = [], [], [], [], [], []
        for li, (a, b) in enumerate(segs):
            pa, pb = project(T, a), project(T, b)
            if pa is None or pb is None:
                continue
            idx = len(ll)
            ll.append(np.array([pa[0][0], pa[0][1], pb[0][0], pb[0][1]]) + rng.normal(0, pixel_sigma, 4))
            stereo = pa[0][2] > 0 and pb[0][2] > 0 and rng.uniform() < 0.6
            lr.append(np.array([pa[0][2], pa[0][1], pb[0][2], pb[0][1]]) + rng.normal(0, pixel_sigma, 4)
                      if stereo else np.zeros(4))
            lv.append(1 if stereo else 0)
            pol.append({kp_of_point[j]: float(rng.uniform(0.1, 1.5)) for j, l2 in line_of_point.items()
                        if l2 == li and j in kp_of_point})
            lobs.append((li, idx))
            if li not in created_l:
                created_l.add(li)
                d = b - a
                d = d / np.linalg.norm(d)
                pc = a + rng.normal(0, 0.03, 3)
                dd = d + rng.normal(0, 0.01, 3)
                dd /= np.linalg.norm(dd)
                newl.append((li, np.concatenate([np.cross(pc, dd), dd])))
        kfs.append(dict(id=k * frames_per_keyframe, timestamp=ts[k], parent_id=(k - 1) * frames_per_keyframe if k else -1,
                        Twc=tracked[k], keypoints=np.array(kps).reshape(-1, 3),
                        lines_left=np.array(ll).reshape(-1, 4), lines_right=np.array(lr).reshape(-1, 4),
                        lines_right_valid=np.array(lv, np.uint8), points_on_lines=pol,
                        new_points=newp, new_lines=newl, point_obs=pobs, line_obs=lobs))
    return dict(camera=np.array(cam, np.float64), gt_Twc=np.array(gt), timestamps=np.array(ts), keyframes=kfs)


def line_scene(n_lines: int = 60, n_points: int = 400, seed: int = 0, width: int = 752, height: int = 480,
               disparity: float = 14.0, frag: int = 3, on_line_frac: float = 0.5, noise: float = 0.4):
    """A stereo frame of the line front end: long scene segments observed as
    FLD-like fragments (each split into `frag` pieces with small gaps, endpoint jitter, on the
    half-size image as fld->detect returns them), keypoints half on / near the segments, half
    anywhere, as the 259-double records' (x, y) rows, and stereo matches (left i <-> its right
    counterpart, shifted by the disparity; a few wrong ones).  Returns a dict of
    seg_left/seg_right [n][4] float32, feat_left/feat_right [N][259], stereo_matches [m][2],
    lines_left/lines_right [n_lines][4] (the full-size scene segments)."""
    rng = np.random.default_rng(seed)
    L = []
    for _ in range(n_lines):
        length = rng.uniform(70, 260)
        a = rng.uniform(-np.pi, np.pi)
        cx, cy = rng.uniform(40, width - 40), rng.uniform(40, height - 40)
        d = np.array([np.cos(a), np.sin(a)]) * length / 2
        p, q = np.clip([cx, cy] - d, 2, [width - 3, height - 3]), np.clip([cx, cy] + d, 2, [width - 3, height - 3])
        if np.hypot(*(q - p)) < 40:
            continue
        L.append(np.concatenate([p, q]))
    L = np.array(L)

    def fragments(lines, shift):
        out = []
        for ln in lines:
            p, q = ln[:2] - [shift, 0], ln[2:] - [shift, 0]
            cuts = np.sort(rng.uniform(0.15, 0.85, frag - 1))
            ts = np.concatenate([[0.0], cuts, [1.0]])
            for k in range(frag):
                t0 = ts[k] + (0.01 if k else 0.0)
                t1 = ts[k + 1] - (0.01 if k < frag - 1 else 0.0)
                a_, b_ = p + (q - p) * t0, p + (q - p) * t1
                jit = rng.normal(0, 0.3, 4)
                seg = (np.concatenate([a_, b_]) + jit) / 2.0
                if rng.random() < 0.5:
                    seg = seg[[2, 3, 0, 1]]
                out.append(seg)
        return np.array(out, np.float32).reshape(-1, 4)

    def points(lines):
        P = []
        n_on = int(n_points * on_line_frac)
        for _ in range(n_on):
            ln = lines[rng.integers(len(lines))]
            t = rng.uniform(-0.03, 1.03)
            off = rng.normal(0, 2.5)
            dirv = ln[2:] - ln[:2]
            nrm = np.array([-dirv[1], dirv[0]]) / np.hypot(*dirv)
            P.append(ln[:2] + dirv * t + nrm * off)
        P += list(np.column_stack([rng.uniform(8, width - 8, n_points - n_on),
                                   rng.uniform(8, height - 8, n_points - n_on)]))
        return np.round(np.array(P), 0)  # SuperPoint keypoints are integer pixels

    xy_left = points(L)
    xy_right = xy_left - [disparity, 0] + np.round(rng.normal(0, noise, xy_left.shape))
    perm = rng.permutation(len(xy_right))
    xy_right = xy_right[perm]
    inv = np.argsort(perm)
    m = np.column_stack([np.arange(len(xy_left)), inv])
    keep = rng.random(len(m)) < 0.8
    m = m[keep]
    wrong = rng.random(len(m)) < 0.05
    m[wrong, 1] = rng.integers(0, len(xy_right), int(wrong.sum()))

    def feats(xy):
        F = np.zeros((len(xy), 259))
        F[:, 0] = rng.uniform(0.01, 1, len(xy))
        F[:, 1:3] = xy
        F[:, 3:] = rng.normal(0, 1, (len(xy), 256)) / 16
        return F

    Lr = L - [disparity, 0, disparity, 0]
    return {"seg_left": fragments(L, 0.0), "seg_right": fragments(L, disparity),
            "feat_left": feats(xy_left), "feat_right": feats(xy_right),
            "stereo_matches": m.astype(np.int32), "lines_left": L, "lines_right": Lr}


def edge_stereo_pair(h: int, w: int, seed: int, n_lines: int = 40, disparity: int = 12):
    """Left / right RCF-like edge images of one stereo frame (the u8 maps the reference's line thread runs
    FLD on, map_builder.cc:285-290, 325-337): an edge_map of width w + disparity, the right view shifted by
    the disparity, as stereo_pair does for the texture."""
    img, _ = edge_map(h, w + disparity, n_lines=n_lines, seed=seed)
    return np.ascontiguousarray(img[:, disparity:]), np.ascontiguousarray(img[:, :w])


def edge_map(h: int = 480, w: int = 752, n_lines: int = 40, seed: int = 0, width: float = 1.2, noise: float = 6.0):
    """An RCF-like edge-probability image (the u8 map LineDetector::LineExtractor runs FLD on,
    map_builder.cc:286): n_lines straight ridges with a Gaussian cross-profile (sigma `width` px,
    peak 180..255) on a dark, noisy background, plus a few blobs.  Returns (image u8 [h][w],
    segments [n][4] float64 -- the ridges' centre lines at full size)."""
    rng = np.random.default_rng(seed)
    img = rng.normal(12.0, noise, (h, w))
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    segs = []
    for _ in range(n_lines):
        length = rng.uniform(60, 300)
        a = rng.uniform(-np.pi, np.pi)
        cx, cy = rng.uniform(30, w - 30), rng.uniform(30, h - 30)
        d = np.array([np.cos(a), np.sin(a)]) * length / 2
        p = np.clip(np.array([cx, cy]) - d, 8, [w - 9, h - 9])
        q = np.clip(np.array([cx, cy]) + d, 8, [w - 9, h - 9])
        v = q - p
        L2 = float(v @ v)
        if L2 < 40.0 ** 2:
            continue
        x0, x1 = int(max(min(p[0], q[0]) - 6, 0)), int(min(max(p[0], q[0]) + 7, w))
        y0, y1 = int(max(min(p[1], q[1]) - 6, 0)), int(min(max(p[1], q[1]) + 7, h))
        X, Y = xx[y0:y1, x0:x1], yy[y0:y1, x0:x1]
        t = np.clip(((X - p[0]) * v[0] + (Y - p[1]) * v[1]) / L2, 0.0, 1.0)
        dist2 = (X - p[0] - t * v[0]) ** 2 + (Y - p[1] - t * v[1]) ** 2
        peak = rng.uniform(180, 255)
        img[y0:y1, x0:x1] = np.maximum(img[y0:y1, x0:x1], peak * np.exp(-dist2 / (2 * width * width)))
        segs.append(np.concatenate([p, q]))
    for _ in range(6):
        bx, by, br = rng.uniform(20, w - 20), rng.uniform(20, h - 20), rng.uniform(3, 9)
        img = np.maximum(img, 200.0 * np.exp(-((xx - bx) ** 2 + (yy - by) ** 2) / (2 * br * br)))
    return np.clip(np.rint(img), 0, 255).astype(np.uint8), np.array(segs, np.float64).reshape(-1, 4)

