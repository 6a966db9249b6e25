"""ORACLE (test infrastructure only): a plain-Python restatement of the reference's map-side local
BA -- Map::LocalMapOptimization and the bookkeeping around it -- used to check librspl's
csrc/map.cpp (the product), never called by it.

Restated from (file:line of /root/reference):
  src/map.cc:121-177   Map::UppdateMapline (line endpoints from the map points on the line)
  src/map.cc:471-525   Map::SearchNeighborFrames (9-frame window from the covisibility graph)
  src/map.cc:527-535   Map::AddFrameVertex
  src/map.cc:537-808   Map::LocalMapOptimization (selection, LocalmapOptimization, outliers, write-back)
  src/map.cc:810-895   Map::MakeFramePair, RemoveOutliers, RemoveLineOutliers
  src/map.cc:897-937   Map::UpdateFrameConnection
  src/map.cc:1007-1024 Map::SaveKeyframeTrajectory
  src/frame.cc:214-219, 372-405, 448-531; src/mappoint.cc; src/mapline.cc (accessors, observers,
  covisibility sets).
Objects hold references like the reference's shared_ptrs.  Equal covisibility weights are
ordered by frame id (the reference: by FramePtr address = allocation order, which is id order
when keyframes are created in sequence).  The BA itself is the oracle's fp64 g2o restatement
(oracle.ba_local).  Parity of this file with the reference C++ is unpinned (no reference test
holds map vectors; the reference C++ is unbuildable here); it is pinned only by reading.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np

UNTRI, GOOD, BAD = 0, 1, 2


class Frame:
    def __init__(self, fid, ts, Twc, kp, ll=None, lr=None, lrv=None, pol=None, parent=None):
        self.id, self.ts = fid, ts
        self.pose = np.array(Twc, np.float64).reshape(4, 4).copy()
        self.kp = np.array(kp, np.float64).reshape(-1, 3)
        self.mappoints: List[Optional[Mappoint]] = [None] * len(self.kp)
        n = 0 if ll is None else len(ll)
        self.lines = [np.array(x, np.float64) for x in (ll if n else [])]
        self.lines_right = [np.array(x, np.float64) for x in (lr if (n and lr is not None) else np.zeros((n, 4)))]
        self.lines_right_valid = [bool(x) for x in (lrv if (n and lrv is not None) else np.zeros(n))]
        self.maplines: List[Optional[Mapline]] = [None] * n
        self.points_on_lines = [dict(d) for d in (pol if pol is not None else [{} for _ in range(n)])]
        self.connections: Dict[int, int] = {}          # frame id -> weight (reference: FramePtr -> weight)
        self.ordered = set()                          # (weight, frame id)
        self.parent = parent
        self.lmo = -1
        self.lmo_fix = -1

    # frame.cc:458-477
    def AddConnection(self, other, w):
        if other.id not in self.connections or self.connections[other.id] != w:
            if other.id in self.connections:
                self.ordered.discard((self.connections[other.id], other.id))
            self.connections[other.id] = w
            self.ordered.add((w, other.id))

    def SetConnections(self, s):
        self.ordered = set(s)
        self.connections = {f: w for w, f in s}

    # frame.cc:513-526
    def DecreaseWeight(self, other, w):
        if other.id not in self.connections:
            return
        ow = self.connections[other.id]
        self.ordered.discard((ow, other.id))
        if (ow < w + 5 and len(self.connections) >= 2) or ow <= w:
            del self.connections[other.id]
        else:
            self.connections[other.id] = ow - w
            self.ordered.add((ow - w, other.id))

    def GetOrderedConnections(self):  # ascending
        return sorted(self.ordered)


class Mappoint:
    def __init__(self, mid, p, type_=GOOD):
        self.id, self.p, self.type = mid, np.array(p, np.float64).copy(), type_
        self.obs: Dict[int, int] = {}
        self.lmo = -1

    def num_obs(self):
        return sum(1 for v in self.obs.values() if v >= 0)


class Mapline:
    def __init__(self, lid, L, type_=GOOD):
        self.id, self.L, self.type = lid, np.array(L, np.float64).copy(), type_
        self.obs: Dict[int, int] = {}
        self.lmo = -1
        self.endpoints = np.zeros(6)
        self.endpoints_valid = False

    def num_obs(self):
        return sum(1 for v in self.obs.values() if v >= 0)


def quat_from_R(R):
    """Eigen Quaterniond(Matrix3d) -> (x, y, z, w)."""
    t = R[0, 0] + R[1, 1] + R[2, 2]
    q = [0.0, 0.0, 0.0, 0.0]
    if t > 0:
        t = math.sqrt(t + 1.0)
        q[3] = 0.5 * t
        t = 0.5 / t
        q[0] = (R[2, 1] - R[1, 2]) * t
        q[1] = (R[0, 2] - R[2, 0]) * t
        q[2] = (R[1, 0] - R[0, 1]) * t
    else:
        i = 0
        if R[1, 1] > R[0, 0]:
            i = 1
        if R[2, 2] > R[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = math.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0)
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (R[k, j] - R[j, k]) * t
        q[j] = (R[j, i] + R[i, j]) * t
        q[k] = (R[k, i] + R[i, k]) * t
    return np.array(q)


def R_from_quat(q):
    x, y, z, w = q
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    return np.array([[1 - (ty * y + tz * z), tx * y - tz * w, tx * z + ty * w],
                     [tx * y + tz * w, 1 - (tx * x + tz * z), ty * z - tx * w],
                     [tx * z - ty * w, ty * z + tx * w, 1 - (tx * x + ty * y)]])


class Map:
    def __init__(self, camera, th=(50.0, 75.0, 50.0, 75.0), iterations=(10, 5)):
        self.camera = np.array(camera, np.float64)
        self.th, self.iterations = th, iterations
        self.keyframes: Dict[int, Frame] = {}
        self.keyframe_ids: List[int] = []
        self.mappoints: Dict[int, Mappoint] = {}
        self.maplines: Dict[int, Mapline] = {}
        self.last = None

    def insert_keyframe(self, f: Frame):
        self.keyframes[f.id] = f
        self.keyframe_ids.append(f.id)

    def add_point_obs(self, pid, fid, k):
        m, f = self.mappoints[pid], self.keyframes[fid]
        m.obs[fid] = k
        f.mappoints[k] = m

    def add_line_obs(self, lid, fid, k):
        l, f = self.maplines[lid], self.keyframes[fid]
        l.obs[fid] = k
        f.maplines[k] = l

    # map.cc:897-937
    def update_frame_connection(self, frame: Frame):
        conns: Dict[int, int] = {}
        for m in frame.mappoints:
            if m is None or m.type == BAD:
                continue
            for oid in m.obs:
                if oid == frame.id or oid not in self.keyframes:
                    continue
                conns[oid] = conns.get(oid, 0) + 1
        if not conns:
            return
        good, best, best_w = set(), None, -1
        for oid in sorted(conns):
            w = conns[oid]
            other = self.keyframes[oid]
            if w > best_w:
                best, best_w = other, w
            if w > 15:
                good.add((w, oid))
                other.AddConnection(frame, w)
        if not good:
            good.add((best_w, best.id))
            best.AddConnection(frame, best_w)
        frame.SetConnections(good)

    # map.cc:471-525
    def search_neighbor_frames(self, frame: Frame) -> List[Frame]:
        target, fid = 9, frame.id
        if len(self.keyframes) <= target:
            out = []
            for k in sorted(self.keyframes):
                self.keyframes[k].lmo = fid
                out.append(self.keyframes[k])
            return out
        out = [frame]
        frame.lmo = fid
        cs = frame.GetOrderedConnections()
        for w, oid in cs[:min(len(cs), target - 1)]:
            o = self.keyframes[oid]
            o.lmo = fid
            out.append(o)
        par = self.keyframes.get(frame.parent) if frame.parent is not None else None
        if par is not None and par.lmo != fid:
            par.lmo = fid
            out.append(par)
        while len(out) < target:
            deeper: Dict[int, int] = {}
            for k in out:
                for w, oid in k.GetOrderedConnections():
                    if self.keyframes[oid].lmo != fid:
                        deeper[oid] = deeper.get(oid, 0) + w
            if not deeper:
                break
            ordered = sorted(((s, oid) for oid, s in deeper.items()), reverse=True)
            for s, oid in ordered[:min(target - len(out), len(ordered))]:
                o = self.keyframes[oid]
                o.lmo = fid
                out.append(o)
        return out

    # map.cc:537-707 -> the LocalmapOptimization inputs
    def assemble(self, fid):
        frame = self.keyframes[fid]
        self.update_frame_connection(frame)
        poses = {}

        def add_vertex(f, fixed):
            if f.id not in poses:
                poses[f.id] = (quat_from_R(f.pose[:3, :3]), f.pose[:3, 3].copy(), fixed)

        nb = self.search_neighbor_frames(frame)
        nfixed = 0
        for k in nb:
            fx = k.id == 0
            nfixed += fx
            add_vertex(k, fx)
        fixed_frames: Dict[int, int] = {}
        mpts, mpls = [], []
        for k in nb:
            for m in k.mappoints:
                if m is None or m.type != GOOD or m.lmo == fid:
                    continue
                m.lmo = fid
                mpts.append(m)
                for oid in m.obs:
                    o = self.keyframes.get(oid)
                    if o is not None and o.lmo != fid:
                        fixed_frames[oid] = fixed_frames.get(oid, 0) + 1
            for l in k.maplines:
                if l is None or l.type != GOOD or l.lmo == fid:
                    continue
                l.lmo = fid
                mpls.append(l)
        if fixed_frames and 1 > nfixed:
            ordered = sorted(((c, oid) for oid, c in fixed_frames.items()), reverse=True)
            for c, oid in ordered[:min(1 - nfixed, len(ordered))]:
                o = self.keyframes[oid]
                o.lmo_fix = fid
                add_vertex(o, True)
        inwin = lambda o: o is not None and (o.lmo == fid or o.lmo_fix == fid)
        cons = {"mono": [], "stereo": [], "mono_line": [], "stereo_line": []}
        points, lines = {}, {}
        for m in mpts:
            if m.type != GOOD:
                continue
            mono, stereo = [], []
            for oid in sorted(m.obs):
                o = self.keyframes.get(oid)
                k = m.obs[oid]
                if not inwin(o) or not (0 <= k < len(o.kp)):
                    continue
                kp = o.kp[k]
                if kp[2] > 0:
                    stereo.append((oid, m.id, kp.copy()))
                else:
                    mono.append((oid, m.id, kp[:2].copy()))
            if stereo or len(mono) > 1:
                points[m.id] = m.p.copy()
                cons["mono"] += mono
                cons["stereo"] += stereo
        for l in mpls:
            if l.type != GOOD:
                continue
            mono, stereo = [], []
            for oid in sorted(l.obs):
                o = self.keyframes.get(oid)
                k = l.obs[oid]
                if not inwin(o) or not (0 <= k < len(o.lines)):
                    continue
                if o.lines_right_valid[k]:
                    stereo.append((oid, l.id, np.concatenate([o.lines[k], o.lines_right[k]])))
                else:
                    mono.append((oid, l.id, o.lines[k].copy()))
            if stereo or len(mono) > 1:
                lines[l.id] = l.L.copy()
                cons["mono_line"] += mono
                cons["stereo_line"] += stereo
        self.last = (fid, poses, points, lines, cons)
        return self.last

    def dense_problem(self):
        """The assembled problem in the C ABI's dense layout (ids ascending, constraints in order)."""
        fid, poses, points, lines, cons = self.last
        pk, qk, lk = sorted(poses), sorted(points), sorted(lines)
        pidx = {k: i for i, k in enumerate(pk)}
        qidx = {k: i for i, k in enumerate(qk)}
        lidx = {k: i for i, k in enumerate(lk)}
        dims = {"mono": 2, "stereo": 3, "mono_line": 4, "stereo_line": 8}
        out = dict(pose_ids=np.array(pk, np.int32), pose_fixed=np.array([poses[k][2] for k in pk], np.uint8),
                   pose_q=np.array([poses[k][0] for k in pk]).reshape(-1, 4),
                   pose_p=np.array([poses[k][1] for k in pk]).reshape(-1, 3),
                   point_ids=np.array(qk, np.int32), points=np.array([points[k] for k in qk]).reshape(-1, 3),
                   line_ids=np.array(lk, np.int32), lines=np.array([lines[k] for k in lk]).reshape(-1, 6))
        for name, cs in cons.items():
            lm = qidx if name in ("mono", "stereo") else lidx
            out[name] = dict(pose=np.array([pidx[c[0]] for c in cs], np.int32),
                             lm=np.array([lm[c[1]] for c in cs], np.int32),
                             obs=np.array([c[2] for c in cs], np.float64).reshape(-1, dims[name]))
        return out

    # map.cc:818-863
    def remove_outliers(self, outliers):
        bad: Dict[tuple, int] = {}
        for f, m in outliers:
            if f is None or m is None or m.type == BAD:
                continue
            m.obs.pop(f.id, None)
            obs = dict(m.obs)
            for oid in obs:
                if oid in self.keyframes:
                    key = (max(f.id, oid), min(f.id, oid))
                    bad[key] = bad.get(key, 0) + 1
            if m.num_obs() < 2 and m.type != BAD:
                delete = True
                if m.num_obs() > 0:
                    first = min(obs)
                    o = self.keyframes.get(first)
                    if o is not None:
                        k = m.obs.get(first, -1)
                        if 0 <= k < len(o.kp) and o.kp[k][2] < 0:
                            slot = obs[first]
                            if 0 <= slot < len(o.mappoints):
                                o.mappoints[slot] = None
                        else:
                            delete = False
                if delete:
                    m.type = BAD
                    m.obs.clear()
            # frame->RemoveMappoint(mpt): looks up the just-removed observer -> index -1 -> no-op
        for (a, b), w in bad.items():
            self.keyframes[a].DecreaseWeight(self.keyframes[b], w)
            self.keyframes[b].DecreaseWeight(self.keyframes[a], w)

    # map.cc:865-895
    def remove_line_outliers(self, outliers):
        for f, l in outliers:
            if f is None or l is None or l.type == BAD:
                continue
            l.obs.pop(f.id, None)
            obs = dict(l.obs)
            if l.num_obs() < 2 and l.type != BAD:
                delete = True
                if l.num_obs() > 0:
                    first = min(obs)
                    o = self.keyframes.get(first)
                    if o is not None:
                        idx = l.obs.get(first, -1)
                        if not (0 <= idx < len(o.lines_right_valid) and o.lines_right_valid[idx]):
                            slot = obs[first]
                            if 0 <= slot < len(o.maplines):
                                o.maplines[slot] = None
                        else:
                            delete = False
                if delete:
                    l.type = BAD
                    l.obs.clear()

    # map.cc:121-177
    def update_mapline(self, l: Mapline) -> bool:
        if l.type != GOOD or not l.obs:
            return False
        pts = []
        for fid in sorted(l.obs):
            f = self.keyframes.get(fid)
            if f is None:
                continue
            k = l.obs[fid]
            if not (0 <= k < len(f.points_on_lines)):
                continue
            for kp in sorted(f.points_on_lines[k]):
                if not (0 <= kp < len(f.mappoints)):
                    continue
                m = f.mappoints[kp]
                if m is not None and m.type == GOOD:
                    pts.append(m.p.copy())
        w, d = l.L[:3], l.L[3:]
        v = d / np.linalg.norm(d)
        W = -np.array([[0, -d[2], d[1]], [d[2], 0, -d[0]], [-d[1], d[0], 0]])
        lp = np.linalg.solve(W.T @ W + 1e-9 * np.eye(3), W.T @ w)     # g2o Line3D::toCartesian
        md = int(np.argmax(np.abs(v)))
        mx, mn, fmax, fmin = 2.2250738585072014e-308, 1.7976931348623157e308, False, False
        for p in pts:
            if np.linalg.norm(np.cross(v, p - lp)) > 0.2:
                continue
            if p[md] > mx:
                mx, fmax = p[md], True
            if p[md] < mn:
                mn, fmin = p[md], True
        if not (fmax and fmin):
            return False
        r1, r2 = (mx - lp[md]) / v[md], (mn - lp[md]) / v[md]
        l.endpoints = np.concatenate([lp + r1 * v, lp + r2 * v])
        l.endpoints_valid = True
        return True

    # map.cc:709-802, with the BA result supplied (dense ids as dense_problem)
    def finish(self, res):
        fid, poses, points, lines, cons = self.last
        pk, qk, lk = sorted(poses), sorted(points), sorted(lines)
        outl, loutl = [], []
        for name in ("mono", "stereo"):
            for c, f in zip(cons[name], res.inlier[name]):
                if not f and c[0] in self.keyframes and c[1] in self.mappoints:
                    outl.append((self.keyframes[c[0]], self.mappoints[c[1]]))
        for name in ("mono_line", "stereo_line"):
            for c, f in zip(cons[name], res.inlier[name]):
                if not f and c[0] in self.keyframes and c[1] in self.maplines:
                    loutl.append((self.keyframes[c[0]], self.maplines[c[1]]))
        self.remove_outliers(outl)
        self.remove_line_outliers(loutl)
        self.update_frame_connection(self.keyframes[fid])
        for i, k in enumerate(pk):
            if k in self.keyframes:
                T = np.eye(4)
                T[:3, :3] = R_from_quat(res.pose_q[i])
                T[:3, 3] = res.pose_p[i]
                self.keyframes[k].pose = T
        for i, k in enumerate(qk):
            if k in self.mappoints:
                self.mappoints[k].p = res.points[i].copy()
        for i, k in enumerate(lk):
            if k in self.maplines:
                l = self.maplines[k]
                l.L = res.lines[i].copy()
                if l.type == UNTRI:
                    l.type = GOOD
                l.endpoints_valid = self.update_mapline(l)
        return len(outl), len(loutl)

    # map.cc:1007-1024
    def trajectory_lines(self):
        out = []
        for fid in self.keyframe_ids:
            f = self.keyframes[fid]
            q = quat_from_R(f.pose[:3, :3])
            t = f.pose[:3, 3]
            out.append("%.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f" % (f.ts, t[0], t[1], t[2], q[0], q[1], q[2], q[3]))
        return out


def insert_keyframe(mr: Map, kf: dict):
    """Oracle side of sequence.insert_keyframe (Map::InsertKeyframe bookkeeping)."""
    f = Frame(kf["id"], kf["timestamp"], kf["Twc"], kf["keypoints"], kf["lines_left"], kf["lines_right"],
              kf["lines_right_valid"], kf["points_on_lines"], kf["parent_id"] if kf["parent_id"] >= 0 else None)
    mr.insert_keyframe(f)
    for i, p in kf["new_points"]:
        mr.mappoints[i] = Mappoint(i, p)
    for i, L in kf["new_lines"]:
        mr.maplines[i] = Mapline(i, L)
    for i, j in kf["point_obs"]:
        mr.add_point_obs(i, kf["id"], j)
    for i, j in kf["line_obs"]:
        mr.add_line_obs(i, kf["id"], j)


def dense_to_problem(d, camera, th, iterations):
    """map_ref.Map.dense_problem -> rspl_slam_amd.ba_types.DenseProblem (for oracle.ba_local)."""
    from rspl_slam_amd.ba_types import DenseProblem, OptimizationConfig
    cfg = OptimizationConfig(mono_point=th[0], stereo_point=th[1], mono_line=th[2], stereo_line=th[3])
    return DenseProblem(cameras=np.array([camera]), pose_q=d["pose_q"], pose_p=d["pose_p"], pose_fixed=d["pose_fixed"],
                        points=d["points"], lines=d["lines"],
                        mono={k: d["mono"][k] for k in ("pose", "lm", "obs")},
                        stereo={k: d["stereo"][k] for k in ("pose", "lm", "obs")},
                        mono_line={k: d["mono_line"][k] for k in ("pose", "lm", "obs")},
                        stereo_line={k: d["stereo_line"][k] for k in ("pose", "lm", "obs")},
                        cfg=cfg, iterations_first=iterations[0], iterations_second=iterations[1])


def local_map_optimization(mr: Map, fid: int, ba_local):
    """Map::LocalMapOptimization on the oracle map with the oracle BA (ba_local = oracle.ba_local)."""
    mr.assemble(fid)
    prob = dense_to_problem(mr.dense_problem(), mr.camera, mr.th, mr.iterations)
    res = ba_local(prob)
    n_out, n_lout = mr.finish(res)
    return prob, res, n_out, n_lout
