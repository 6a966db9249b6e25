"""Host-side mirror of the reference's BA data model and its C-ABI marshalling.

Reference: include/g2o_optimization/types.h:19-174 (Pose3d, Position3d, Line3d,
Mono/Stereo Point/Line constraints), include/read_configs.h:50-56
(OptimizationConfig).  The reference keys vertices by id in std::maps; the C ABI
(include/rspl.h, rspl_ba_problem) takes dense arrays, so ``pack_problem``
remaps ids to dense indices exactly once per call.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np


@dataclass
class Pose3d:                      # types.h:19-33 (T_wc)
    fixed: bool
    p: np.ndarray                  # [3]
    q: np.ndarray                  # [4] Eigen coeffs order (x, y, z, w)


@dataclass
class Position3d:                  # types.h:38-50
    fixed: bool
    p: np.ndarray


@dataclass
class Line3d:                      # types.h:108-120 (g2o::Line3D Pluecker (w, d))
    fixed: bool
    line_3d: np.ndarray            # [6]


@dataclass
class MonoPointConstraint:         # types.h:54-78
    id_pose: int
    id_point: int
    id_camera: int
    keypoint: np.ndarray           # [2]
    inlier: bool = True
    pixel_sigma: float = 0.8


@dataclass
class StereoPointConstraint:       # types.h:81-105
    id_pose: int
    id_point: int
    id_camera: int
    keypoint: np.ndarray           # [3] u, v, u_right
    inlier: bool = True
    pixel_sigma: float = 0.8


@dataclass
class MonoLineConstraint:          # types.h:124-148
    id_pose: int
    id_line: int
    id_camera: int
    line_2d: np.ndarray            # [4]
    inlier: bool = True
    pixel_sigma: float = 0.8


@dataclass
class StereoLineConstraint:        # types.h:151-174
    id_pose: int
    id_line: int
    id_camera: int
    line_2d: np.ndarray            # [8]
    inlier: bool = True
    pixel_sigma: float = 0.8


@dataclass
class Camera:                      # include/camera.h:25-29 accessors used by the BA
    fx: float
    fy: float
    cx: float
    cy: float
    bf: float


@dataclass
class OptimizationConfig:          # include/read_configs.h:50-56 (configs_euroc.yaml:56-61)
    mono_point: float = 50.0
    stereo_point: float = 75.0
    mono_line: float = 50.0
    stereo_line: float = 75.0
    rate: float = 0.5


class RsplBaProblem(C.Structure):
    _fields_ = [
        ("n_cameras", C.c_int), ("cameras", C.POINTER(C.c_double)),
        ("n_poses", C.c_int), ("pose_q", C.POINTER(C.c_double)), ("pose_p", C.POINTER(C.c_double)),
        ("pose_fixed", C.POINTER(C.c_uint8)),
        ("n_points", C.c_int), ("points", C.POINTER(C.c_double)),
        ("n_lines", C.c_int), ("lines", C.POINTER(C.c_double)),
        ("n_mono", C.c_int), ("mono_pose", C.POINTER(C.c_int32)), ("mono_point", C.POINTER(C.c_int32)),
        ("mono_camera", C.POINTER(C.c_int32)), ("mono_obs", C.POINTER(C.c_double)),
        ("n_stereo", C.c_int), ("stereo_pose", C.POINTER(C.c_int32)), ("stereo_point", C.POINTER(C.c_int32)),
        ("stereo_camera", C.POINTER(C.c_int32)), ("stereo_obs", C.POINTER(C.c_double)),
        ("n_mono_line", C.c_int), ("mono_line_pose", C.POINTER(C.c_int32)),
        ("mono_line_line", C.POINTER(C.c_int32)), ("mono_line_camera", C.POINTER(C.c_int32)),
        ("mono_line_obs", C.POINTER(C.c_double)),
        ("n_stereo_line", C.c_int), ("stereo_line_pose", C.POINTER(C.c_int32)),
        ("stereo_line_line", C.POINTER(C.c_int32)), ("stereo_line_camera", C.POINTER(C.c_int32)),
        ("stereo_line_obs", C.POINTER(C.c_double)),
        ("th_mono_point", C.c_double), ("th_stereo_point", C.c_double),
        ("th_mono_line", C.c_double), ("th_stereo_line", C.c_double),
        ("iterations_first", C.c_int), ("iterations_second", C.c_int),
    ]


class RsplBaResult(C.Structure):  # output pointers as plain addresses (set from one result buffer)
    _fields_ = [
        ("pose_q", C.c_void_p), ("pose_p", C.c_void_p),
        ("points", C.c_void_p), ("lines", C.c_void_p),
        ("mono_inlier", C.c_void_p), ("stereo_inlier", C.c_void_p),
        ("mono_line_inlier", C.c_void_p), ("stereo_line_inlier", C.c_void_p),
        ("chi2_first", C.c_double), ("chi2_second", C.c_double),
        ("iterations_done_first", C.c_int), ("iterations_done_second", C.c_int),
    ]


def _ptr(a, ct):
    if a is None:
        return C.POINTER(ct)()
    return a.ctypes.data_as(C.POINTER(ct))


@dataclass
class DenseProblem:
    """Dense-index arrays of one LocalmapOptimization call (C-ABI rspl_ba_problem)."""
    cameras: np.ndarray                          # [nc, 5]
    pose_q: np.ndarray                           # [np, 4] (x, y, z, w) of T_wc
    pose_p: np.ndarray                           # [np, 3]
    pose_fixed: np.ndarray                       # [np] uint8
    points: np.ndarray                           # [nq, 3]
    lines: np.ndarray                            # [nl, 6]
    mono: Dict[str, np.ndarray] = field(default_factory=dict)     # pose, lm, cam, obs
    stereo: Dict[str, np.ndarray] = field(default_factory=dict)
    mono_line: Dict[str, np.ndarray] = field(default_factory=dict)
    stereo_line: Dict[str, np.ndarray] = field(default_factory=dict)
    cfg: OptimizationConfig = field(default_factory=OptimizationConfig)
    iterations_first: int = 10
    iterations_second: int = 5

    def __post_init__(self):
        f = lambda a, dt: np.ascontiguousarray(a, dtype=dt)
        self.cameras = f(self.cameras, np.float64).reshape(-1, 5)
        self.pose_q = f(self.pose_q, np.float64).reshape(-1, 4)
        self.pose_p = f(self.pose_p, np.float64).reshape(-1, 3)
        self.pose_fixed = f(self.pose_fixed, np.uint8).reshape(-1)
        self.points = f(self.points, np.float64).reshape(-1, 3)
        self.lines = f(self.lines, np.float64).reshape(-1, 6)
        for name, od in (("mono", 2), ("stereo", 3), ("mono_line", 4), ("stereo_line", 8)):
            d = getattr(self, name)
            n = len(d.get("pose", []))
            d["pose"] = f(d.get("pose", np.zeros(0)), np.int32).reshape(-1)
            d["lm"] = f(d.get("lm", np.zeros(0)), np.int32).reshape(-1)
            d["cam"] = f(d.get("cam", np.zeros(n)), np.int32).reshape(-1)
            d["obs"] = f(d.get("obs", np.zeros((0, od))), np.float64).reshape(-1, od)

    def n_edges(self, name):
        return int(getattr(self, name)["pose"].shape[0])

    _EDGE_SETS = (("mono", "mono", "point"), ("stereo", "stereo", "point"),
                  ("mono_line", "mono_line", "line"), ("stereo_line", "stereo_line", "line"))

    def _arrays(self):
        return (self.cameras, self.pose_q, self.pose_p, self.pose_fixed, self.points, self.lines) + tuple(
            getattr(self, name)[k] for name, _, _ in self._EDGE_SETS for k in ("pose", "lm", "cam", "obs"))

    def to_ctypes(self) -> RsplBaProblem:
        # the pointer struct is rebuilt only when an array object changed (the cache holds the
        # arrays it points into, so they stay alive); counts and scalars are set on every call
        arrays = self._arrays()
        cache = self.__dict__.get("_ct_cache")
        if cache is None or any(a is not b for a, b in zip(cache[0], arrays)):
            P = RsplBaProblem()
            P.cameras = _ptr(self.cameras, C.c_double)
            P.pose_q = _ptr(self.pose_q, C.c_double)
            P.pose_p = _ptr(self.pose_p, C.c_double)
            P.pose_fixed = _ptr(self.pose_fixed, C.c_uint8)
            P.points = _ptr(self.points, C.c_double)
            P.lines = _ptr(self.lines, C.c_double)
            for name, pre, lmname in self._EDGE_SETS:
                d = getattr(self, name)
                setattr(P, f"{pre}_pose", _ptr(d["pose"], C.c_int32))
                setattr(P, f"{pre}_{lmname}", _ptr(d["lm"], C.c_int32))
                setattr(P, f"{pre}_camera", _ptr(d["cam"], C.c_int32))
                setattr(P, f"{pre}_obs", _ptr(d["obs"], C.c_double))
            self.__dict__["_ct_cache"] = cache = (arrays, P)
        P = cache[1]
        P.n_cameras = self.cameras.shape[0]
        P.n_poses = self.pose_q.shape[0]
        P.n_points = self.points.shape[0]
        P.n_lines = self.lines.shape[0]
        for name, pre, _ in self._EDGE_SETS:
            setattr(P, f"n_{pre}", getattr(self, name)["pose"].shape[0])
        P.th_mono_point = self.cfg.mono_point
        P.th_stereo_point = self.cfg.stereo_point
        P.th_mono_line = self.cfg.mono_line
        P.th_stereo_line = self.cfg.stereo_line
        P.iterations_first = self.iterations_first
        P.iterations_second = self.iterations_second
        return P


@dataclass
class DenseResult:
    pose_q: np.ndarray
    pose_p: np.ndarray
    points: np.ndarray
    lines: np.ndarray
    inlier: Dict[str, np.ndarray]
    chi2_first: float = 0.0
    chi2_second: float = 0.0
    iters_first: int = 0
    iters_second: int = 0

    _KINDS = ("mono", "stereo", "mono_line", "stereo_line")

    @staticmethod
    def alloc(p: DenseProblem) -> "DenseResult":
        # one buffer for every output (all entries are written by rspl_ba_local): doubles first,
        # then the inlier flags; the arrays are views, their addresses base + offset
        shapes = [p.pose_q.shape, p.pose_p.shape, p.points.shape, p.lines.shape]
        nd = [int(np.prod(sh)) for sh in shapes]
        ni = [p.n_edges(k) for k in DenseResult._KINDS]
        buf = np.empty(8 * sum(nd) + sum(ni), np.uint8)
        dbl = buf[:8 * sum(nd)].view(np.float64)
        views, offs, o = [], [], 0
        for sh, n in zip(shapes, nd):
            views.append(dbl[o:o + n].reshape(sh))
            offs.append(8 * o)
            o += n
        o8 = 8 * o
        inl = {}
        for k, n in zip(DenseResult._KINDS, ni):
            inl[k] = buf[o8:o8 + n]
            offs.append(o8)
            o8 += n
        r = DenseResult(pose_q=views[0], pose_p=views[1], points=views[2], lines=views[3], inlier=inl)
        r._buf, r._offs = buf, offs
        return r

    def fits(self, p: DenseProblem) -> bool:
        """this result's arrays have the shapes a result of problem p needs"""
        return (self.pose_q.shape == p.pose_q.shape and self.pose_p.shape == p.pose_p.shape and
                self.points.shape == p.points.shape and self.lines.shape == p.lines.shape and
                all(self.inlier[k].shape[0] == p.n_edges(k) for k in DenseResult._KINDS))

    def to_ctypes(self) -> RsplBaResult:
        buf = getattr(self, "_buf", None)
        if buf is not None:
            R = self.__dict__.get("_ct")
            if R is None:  # one pointer struct per buffer (the scalars are rewritten by every call)
                R = RsplBaResult()
                base = buf.ctypes.data
                (R.pose_q, R.pose_p, R.points, R.lines, R.mono_inlier, R.stereo_inlier, R.mono_line_inlier,
                 R.stereo_line_inlier) = (base + o for o in self._offs)
                self.__dict__["_ct"] = R
            return R
        R = RsplBaResult()
        arrs = [self.pose_q, self.pose_p, self.points, self.lines] + [self.inlier[k] for k in self._KINDS]
        (R.pose_q, R.pose_p, R.points, R.lines, R.mono_inlier, R.stereo_inlier, R.mono_line_inlier,
         R.stereo_line_inlier) = (np.ascontiguousarray(a).ctypes.data for a in arrs)
        return R

    def read_back(self, R: RsplBaResult):
        self.chi2_first = R.chi2_first
        self.chi2_second = R.chi2_second
        self.iters_first = R.iterations_done_first
        self.iters_second = R.iterations_done_second


def pack_problem(poses: Dict[int, Pose3d], points: Dict[int, Position3d], lines: Dict[int, Line3d],
                 camera_list: List[Camera], mono: List[MonoPointConstraint], stereo: List[StereoPointConstraint],
                 mono_line: List[MonoLineConstraint], stereo_line: List[StereoLineConstraint],
                 cfg: OptimizationConfig):
    """std::map ids -> dense indices (LocalmapOptimization's vertex id scheme, g2o_optimization.cc:38-70)."""
    pid = {k: i for i, k in enumerate(sorted(poses))}
    qid = {k: i for i, k in enumerate(sorted(points))}
    lid = {k: i for i, k in enumerate(sorted(lines))}
    ps = [poses[k] for k in sorted(poses)]
    cams = np.array([[c.fx, c.fy, c.cx, c.cy, c.bf] for c in camera_list], np.float64)

    def edges(cs, lmap, lattr, oattr, od):
        return dict(pose=np.array([pid[c.id_pose] for c in cs], np.int32),
                    lm=np.array([lmap[getattr(c, lattr)] for c in cs], np.int32),
                    cam=np.array([c.id_camera for c in cs], np.int32),
                    obs=np.array([getattr(c, oattr) for c in cs], np.float64).reshape(-1, od))

    dp = DenseProblem(
        cameras=cams,
        pose_q=np.array([p.q for p in ps]).reshape(-1, 4), pose_p=np.array([p.p for p in ps]).reshape(-1, 3),
        pose_fixed=np.array([p.fixed for p in ps], np.uint8),
        points=np.array([points[k].p for k in sorted(points)]).reshape(-1, 3),
        lines=np.array([lines[k].line_3d for k in sorted(lines)]).reshape(-1, 6),
        mono=edges(mono, qid, "id_point", "keypoint", 2),
        stereo=edges(stereo, qid, "id_point", "keypoint", 3),
        mono_line=edges(mono_line, lid, "id_line", "line_2d", 4),
        stereo_line=edges(stereo_line, lid, "id_line", "line_2d", 8),
        cfg=cfg)
    return dp, (sorted(poses), sorted(points), sorted(lines))


def unpack_result(res: DenseResult, ids, poses, points, lines, mono, stereo, mono_line, stereo_line):
    """Write back in place (g2o_optimization.cc:212-251)."""
    pk, qk, lk = ids
    for i, k in enumerate(pk):
        poses[k].q = res.pose_q[i].copy()
        poses[k].p = res.pose_p[i].copy()
    for i, k in enumerate(qk):
        points[k].p = res.points[i].copy()
    for i, k in enumerate(lk):
        lines[k].line_3d = res.lines[i].copy()
    for cs, name in ((mono, "mono"), (stereo, "stereo"), (mono_line, "mono_line"), (stereo_line, "stereo_line")):
        for c, f in zip(cs, res.inlier[name]):
            c.inlier = bool(f)


# ---------------------------------------------------------------------------
# FrameOptimization (g2o_optimization.cc:256-398): C-ABI rspl_frame_problem / _result
# ---------------------------------------------------------------------------
class RsplFrameProblem(C.Structure):
    _fields_ = [
        ("n_cameras", C.c_int), ("cameras", C.POINTER(C.c_double)),
        ("pose_q", C.c_double * 4), ("pose_p", C.c_double * 3),
        ("n_points", C.c_int), ("points", C.POINTER(C.c_double)),
        ("n_mono", C.c_int), ("mono_point", C.POINTER(C.c_int32)), ("mono_camera", C.POINTER(C.c_int32)),
        ("mono_obs", C.POINTER(C.c_double)), ("mono_inlier_in", C.POINTER(C.c_uint8)),
        ("n_stereo", C.c_int), ("stereo_point", C.POINTER(C.c_int32)), ("stereo_camera", C.POINTER(C.c_int32)),
        ("stereo_obs", C.POINTER(C.c_double)), ("stereo_inlier_in", C.POINTER(C.c_uint8)),
        ("th_mono_point", C.c_double), ("th_stereo_point", C.c_double),
    ]


class RsplFrameResult(C.Structure):
    _fields_ = [
        ("pose_q", C.c_double * 4), ("pose_p", C.c_double * 3),
        ("mono_inlier", C.POINTER(C.c_uint8)), ("stereo_inlier", C.POINTER(C.c_uint8)),
        ("n_inliers", C.c_int), ("rounds", C.c_int), ("iterations", C.c_int * 4), ("chi2", C.c_double * 4),
    ]


@dataclass
class FrameProblem:
    """Dense arrays of one FrameOptimization call (one pose, fixed points, unary edges)."""
    cameras: np.ndarray                          # [nc, 5]
    pose_q: np.ndarray                           # [4] (x, y, z, w) of the initial T_wc
    pose_p: np.ndarray                           # [3]
    points: np.ndarray                           # [nq, 3]
    mono: Dict[str, np.ndarray] = field(default_factory=dict)     # lm, cam, obs, inlier
    stereo: Dict[str, np.ndarray] = field(default_factory=dict)
    cfg: OptimizationConfig = field(default_factory=OptimizationConfig)

    def __post_init__(self):
        f = lambda a, dt: np.ascontiguousarray(a, dtype=dt)
        self.cameras = f(self.cameras, np.float64).reshape(-1, 5)
        self.pose_q = f(self.pose_q, np.float64).reshape(4)
        self.pose_p = f(self.pose_p, np.float64).reshape(3)
        self.points = f(self.points, np.float64).reshape(-1, 3)
        for name, od in (("mono", 2), ("stereo", 3)):
            d = getattr(self, name)
            n = len(d.get("lm", []))
            d["lm"] = f(d.get("lm", np.zeros(0)), np.int32).reshape(-1)
            d["cam"] = f(d.get("cam", np.zeros(n)), np.int32).reshape(-1)
            d["obs"] = f(d.get("obs", np.zeros((0, od))), np.float64).reshape(-1, od)
            d["inlier"] = f(d.get("inlier", np.ones(n)), np.uint8).reshape(-1)

    def n_edges(self, name):
        return int(getattr(self, name)["lm"].shape[0])

    def to_ctypes(self) -> RsplFrameProblem:
        P = RsplFrameProblem()
        P.n_cameras = self.cameras.shape[0]
        P.cameras = _ptr(self.cameras, C.c_double)
        P.pose_q[:] = list(self.pose_q)
        P.pose_p[:] = list(self.pose_p)
        P.n_points = self.points.shape[0]
        P.points = _ptr(self.points, C.c_double)
        for name in ("mono", "stereo"):
            d = getattr(self, name)
            setattr(P, f"n_{name}", d["lm"].shape[0])
            setattr(P, f"{name}_point", _ptr(d["lm"], C.c_int32))
            setattr(P, f"{name}_camera", _ptr(d["cam"], C.c_int32))
            setattr(P, f"{name}_obs", _ptr(d["obs"], C.c_double))
            setattr(P, f"{name}_inlier_in", _ptr(d["inlier"], C.c_uint8))
        P.th_mono_point = self.cfg.mono_point
        P.th_stereo_point = self.cfg.stereo_point
        return P


@dataclass
class FrameResult:
    pose_q: np.ndarray
    pose_p: np.ndarray
    inlier: Dict[str, np.ndarray]
    n_inliers: int = 0
    rounds: int = 0
    iterations: tuple = ()
    chi2: tuple = ()

    @staticmethod
    def alloc(p: FrameProblem) -> "FrameResult":
        return FrameResult(pose_q=np.zeros(4), pose_p=np.zeros(3),
                           inlier={k: np.zeros(p.n_edges(k), np.uint8) for k in ("mono", "stereo")})

    def to_ctypes(self) -> RsplFrameResult:
        R = RsplFrameResult()
        R.mono_inlier = _ptr(self.inlier["mono"], C.c_uint8)
        R.stereo_inlier = _ptr(self.inlier["stereo"], C.c_uint8)
        return R

    def read_back(self, R: RsplFrameResult):
        self.pose_q = np.array(R.pose_q[:])
        self.pose_p = np.array(R.pose_p[:])
        self.n_inliers = R.n_inliers
        self.rounds = R.rounds
        self.iterations = tuple(R.iterations[:])
        self.chi2 = tuple(R.chi2[:])


def pack_frame_problem(poses: Dict[int, Pose3d], points: Dict[int, Position3d], camera_list: List[Camera],
                       mono: List[MonoPointConstraint], stereo: List[StereoPointConstraint],
                       cfg: OptimizationConfig) -> FrameProblem:
    """FrameOptimization's inputs (one pose, asserted at g2o_optimization.cc:259) -> dense arrays."""
    assert len(poses) == 1, "FrameOptimization takes exactly one pose (g2o_optimization.cc:259)"
    pose = next(iter(poses.values()))
    qid = {k: i for i, k in enumerate(sorted(points))}
    cams = np.array([[c.fx, c.fy, c.cx, c.cy, c.bf] for c in camera_list], np.float64)

    def edges(cs, od):
        return dict(lm=np.array([qid[c.id_point] for c in cs], np.int32),
                    cam=np.array([c.id_camera for c in cs], np.int32),
                    obs=np.array([c.keypoint for c in cs], np.float64).reshape(-1, od),
                    inlier=np.array([c.inlier for c in cs], np.uint8))

    return FrameProblem(cameras=cams, pose_q=pose.q, pose_p=pose.p,
                        points=np.array([points[k].p for k in sorted(points)]).reshape(-1, 3),
                        mono=edges(mono, 2), stereo=edges(stereo, 3), cfg=cfg)
