"""Map-side local BA: the reference's Map bookkeeping over the rspl_map_* C ABI.

Mirrors include/map.h:15-52 (Map::InsertKeyframe / InsertMappoint / InsertMapline /
UpdateFrameConnection / LocalMapOptimization / SaveKeyframeTrajectory) with frames, map points
and map lines named by id.  The selection, outlier removal, covisibility bookkeeping and
write-back run in librspl (csrc/map.cpp, C++); the LocalmapOptimization inside
LocalMapOptimization is the GPU BA of a ``LocalBA`` handle.  There is no CPU path.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import capi
from .ba_types import OptimizationConfig

UNTRIANGULATED, GOOD, BAD = 0, 1, 2  # Mappoint::Type / Mapline::Type

_i32p, _u8p, _dp = C.POINTER(C.c_int32), C.POINTER(C.c_uint8), C.POINTER(C.c_double)


class MapConfig(C.Structure):
    _fields_ = [("camera", _dp), ("th_mono_point", C.c_double), ("th_stereo_point", C.c_double),
                ("th_mono_line", C.c_double), ("th_stereo_line", C.c_double),
                ("iterations_first", C.c_int), ("iterations_second", C.c_int)]


class MapKeyframe(C.Structure):
    _fields_ = [("frame_id", C.c_int), ("timestamp", C.c_double), ("Twc", _dp), ("n_keypoints", C.c_int),
                ("keypoints", _dp), ("n_lines", C.c_int), ("lines_left", _dp), ("lines_right", _dp),
                ("lines_right_valid", _u8p), ("pol_offsets", _i32p), ("pol_points", _i32p), ("pol_dist", _dp),
                ("parent_id", C.c_int)]


class MapReport(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("n_poses", "n_fixed", "n_points", "n_lines", "n_mono", "n_stereo",
                                       "n_mono_line", "n_stereo_line", "n_point_outliers", "n_line_outliers")] + \
               [("chi2_first", C.c_double), ("chi2_second", C.c_double),
                ("iterations_first", C.c_int), ("iterations_second", C.c_int),
                ("assembly_us", C.c_double), ("ba_us", C.c_double), ("finish_us", C.c_double)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


def _declare(lib):
    if getattr(lib, "_rspl_map_declared", False):
        return lib
    vp, ip = C.c_void_p, C.c_int
    lib.rspl_map_create.argtypes = [C.POINTER(MapConfig), C.POINTER(vp)]
    lib.rspl_map_destroy.argtypes = [vp]
    lib.rspl_map_destroy.restype = None
    lib.rspl_map_add_keyframe.argtypes = [vp, C.POINTER(MapKeyframe)]
    lib.rspl_map_add_mappoint.argtypes = [vp, ip, _dp, ip]
    lib.rspl_map_add_mapline.argtypes = [vp, ip, _dp, ip]
    lib.rspl_map_add_point_observation.argtypes = [vp, ip, ip, ip]
    lib.rspl_map_add_line_observation.argtypes = [vp, ip, ip, ip]
    lib.rspl_map_add_mappoints.argtypes = [vp, ip, _i32p, _dp, _i32p]
    lib.rspl_map_add_point_observations.argtypes = [vp, ip, ip, _i32p, _i32p]
    lib.rspl_map_update_connections.argtypes = [vp, ip]
    lib.rspl_map_local_optimization.argtypes = [vp, ip, vp, C.POINTER(MapReport)]
    lib.rspl_map_assemble.argtypes = [vp, ip, C.POINTER(MapReport)]
    lib.rspl_map_finish.argtypes = [vp, vp, C.POINTER(MapReport)]
    lib.rspl_map_last_problem.argtypes = [vp, _i32p, _u8p, _i32p, _i32p, C.POINTER(_i32p), C.POINTER(_i32p),
                                          C.POINTER(_dp)]
    lib.rspl_map_get_keyframe.argtypes = [vp, ip, _dp, C.POINTER(ip)]
    lib.rspl_map_get_connections.argtypes = [vp, ip, _i32p, _i32p, ip, C.POINTER(ip)]
    lib.rspl_map_get_mappoint.argtypes = [vp, ip, _dp, C.POINTER(ip), C.POINTER(ip), _i32p, _i32p, ip]
    lib.rspl_map_get_mapline.argtypes = [vp, ip, _dp, C.POINTER(ip), C.POINTER(ip), _dp, C.POINTER(ip)]
    lib.rspl_map_get_frame_slots.argtypes = [vp, ip, _i32p, _i32p]
    lib.rspl_map_save_trajectory.argtypes = [vp, C.c_char_p]
    lib._rspl_map_declared = True
    return lib


def _p(a, ct):
    return a.ctypes.data_as(C.POINTER(ct)) if a is not None else None


OBS_DIMS = (2, 3, 4, 8)  # mono, stereo, mono line, stereo line
KINDS = ("mono", "stereo", "mono_line", "stereo_line")


class Map:
    """Map (include/map.h:15-52) of keyframes, map points and map lines."""

    def __init__(self, camera: Sequence[float], cfg: OptimizationConfig = OptimizationConfig(),
                 iterations=(10, 5)):
        self._lib = _declare(capi.load())
        self._cam = np.ascontiguousarray(camera, np.float64)
        c = MapConfig(_p(self._cam, C.c_double), cfg.mono_point, cfg.stereo_point, cfg.mono_line, cfg.stereo_line,
                      iterations[0], iterations[1])
        self._h = C.c_void_p()
        capi.check(self._lib.rspl_map_create(C.byref(c), C.byref(self._h)), "rspl_map_create")
        self._nkp: Dict[int, int] = {}
        self._nl: Dict[int, int] = {}

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            self._lib.rspl_map_destroy(self._h)
            self._h = C.c_void_p()

    # ---- building (Map::InsertKeyframe / InsertMappoint / InsertMapline bookkeeping) ----
    def InsertKeyframe(self, frame_id: int, timestamp: float, Twc: np.ndarray, keypoints: np.ndarray,
                       lines_left: Optional[np.ndarray] = None, lines_right: Optional[np.ndarray] = None,
                       lines_right_valid: Optional[np.ndarray] = None,
                       points_on_lines: Optional[List[Dict[int, float]]] = None, parent_id: int = -1):
        T = np.ascontiguousarray(Twc, np.float64).reshape(16)
        kp = np.ascontiguousarray(keypoints, np.float64).reshape(-1, 3)
        nl = 0 if lines_left is None else len(lines_left)
        ll = np.ascontiguousarray(lines_left, np.float64).reshape(-1, 4) if nl else None
        lr = np.ascontiguousarray(lines_right, np.float64).reshape(-1, 4) if nl and lines_right is not None else None
        lv = np.ascontiguousarray(lines_right_valid, np.uint8) if nl and lines_right_valid is not None else None
        off = pts = dist = None
        if nl and points_on_lines is not None:
            off = np.zeros(nl + 1, np.int32)
            for i, d in enumerate(points_on_lines):
                off[i + 1] = off[i] + len(d)
            pts = np.array([k for d in points_on_lines for k in sorted(d)], np.int32)
            dist = np.array([d[k] for d in points_on_lines for k in sorted(d)], np.float64)
        k = MapKeyframe(frame_id, timestamp, _p(T, C.c_double), len(kp), _p(kp, C.c_double), nl,
                        _p(ll, C.c_double), _p(lr, C.c_double), _p(lv, C.c_uint8), _p(off, C.c_int32),
                        _p(pts, C.c_int32), _p(dist, C.c_double), parent_id)
        capi.check(self._lib.rspl_map_add_keyframe(self._h, C.byref(k)), "rspl_map_add_keyframe")
        self._nkp[frame_id] = len(kp)
        self._nl[frame_id] = nl

    def InsertMappoint(self, point_id: int, p, type_: int = GOOD):
        a = np.ascontiguousarray(p, np.float64)
        capi.check(self._lib.rspl_map_add_mappoint(self._h, point_id, _p(a, C.c_double), type_),
                   "rspl_map_add_mappoint")

    def InsertMapline(self, line_id: int, line3d, type_: int = GOOD):
        a = np.ascontiguousarray(line3d, np.float64)
        capi.check(self._lib.rspl_map_add_mapline(self._h, line_id, _p(a, C.c_double), type_), "rspl_map_add_mapline")

    def AddPointObservation(self, point_id: int, frame_id: int, keypoint_idx: int):
        capi.check(self._lib.rspl_map_add_point_observation(self._h, point_id, frame_id, keypoint_idx),
                   "rspl_map_add_point_observation")

    def InsertMappoints(self, ids, P, types=None):
        ids = np.ascontiguousarray(ids, np.int32)
        P = np.ascontiguousarray(P, np.float64).reshape(-1, 3)
        t = np.ascontiguousarray(types, np.int32) if types is not None else None
        capi.check(self._lib.rspl_map_add_mappoints(self._h, len(ids), _p(ids, C.c_int32), _p(P, C.c_double),
                                                    _p(t, C.c_int32)), "rspl_map_add_mappoints")

    def AddPointObservations(self, frame_id: int, point_ids, keypoints):
        a = np.ascontiguousarray(point_ids, np.int32)
        b = np.ascontiguousarray(keypoints, np.int32)
        capi.check(self._lib.rspl_map_add_point_observations(self._h, frame_id, len(a), _p(a, C.c_int32),
                                                             _p(b, C.c_int32)), "rspl_map_add_point_observations")

    def AddLineObservation(self, line_id: int, frame_id: int, line_idx: int):
        capi.check(self._lib.rspl_map_add_line_observation(self._h, line_id, frame_id, line_idx),
                   "rspl_map_add_line_observation")

    def UpdateFrameConnection(self, frame_id: int):
        capi.check(self._lib.rspl_map_update_connections(self._h, frame_id), "rspl_map_update_connections")

    # ---- Map::LocalMapOptimization ----
    def LocalMapOptimization(self, frame_id: int, ba) -> dict:
        """The whole of Map::LocalMapOptimization(new_frame) with the GPU local BA of `ba` (LocalBA)."""
        r = MapReport()
        capi.check(self._lib.rspl_map_local_optimization(self._h, frame_id, ba._h, C.byref(r)),
                   "rspl_map_local_optimization")
        return r.as_dict()

    def Assemble(self, frame_id: int) -> dict:
        """Window / constraint selection only (no BA, no write-back)."""
        r = MapReport()
        capi.check(self._lib.rspl_map_assemble(self._h, frame_id, C.byref(r)), "rspl_map_assemble")
        return r.as_dict()

    def LastProblem(self, report: dict) -> dict:
        n = report
        pid = np.zeros(n["n_poses"], np.int32)
        pfx = np.zeros(n["n_poses"], np.uint8)
        qid = np.zeros(n["n_points"], np.int32)
        lid = np.zeros(n["n_lines"], np.int32)
        cnt = [n["n_" + k] for k in KINDS]
        cp = [np.zeros(c, np.int32) for c in cnt]
        cl = [np.zeros(c, np.int32) for c in cnt]
        co = [np.zeros((c, d), np.float64) for c, d in zip(cnt, OBS_DIMS)]
        P = (_i32p * 4)(*[_p(a, C.c_int32) for a in cp])
        L = (_i32p * 4)(*[_p(a, C.c_int32) for a in cl])
        O = (_dp * 4)(*[_p(a, C.c_double) for a in co])
        capi.check(self._lib.rspl_map_last_problem(self._h, _p(pid, C.c_int32), _p(pfx, C.c_uint8), _p(qid, C.c_int32),
                                                   _p(lid, C.c_int32), P, L, O), "rspl_map_last_problem")
        return dict(pose_ids=pid, pose_fixed=pfx, point_ids=qid, line_ids=lid,
                    **{k: dict(pose=a, lm=b, obs=c) for k, a, b, c in zip(KINDS, cp, cl, co)})

    def Finish(self, result) -> dict:
        """Apply a BA result (ba_types.DenseResult) to the last assembled problem: outlier removal,
        covisibility update, write-back (map.cc:712-802)."""
        R = result.to_ctypes()
        r = MapReport()
        capi.check(self._lib.rspl_map_finish(self._h, C.byref(R), C.byref(r)), "rspl_map_finish")
        return r.as_dict()

    # ---- queries ----
    def GetPose(self, frame_id: int) -> np.ndarray:
        T = np.zeros(16)
        capi.check(self._lib.rspl_map_get_keyframe(self._h, frame_id, _p(T, C.c_double), None), "rspl_map_get_keyframe")
        return T.reshape(4, 4)

    def GetOrderedConnections(self, frame_id: int):
        """Frame::GetOrderedConnections(-1): [(weight, frame id)] ascending."""
        n = C.c_int()
        capi.check(self._lib.rspl_map_get_connections(self._h, frame_id, None, None, 0, C.byref(n)),
                   "rspl_map_get_connections")
        ids, ws = np.zeros(n.value, np.int32), np.zeros(n.value, np.int32)
        capi.check(self._lib.rspl_map_get_connections(self._h, frame_id, _p(ids, C.c_int32), _p(ws, C.c_int32),
                                                      n.value, C.byref(n)), "rspl_map_get_connections")
        return [(int(w), int(i)) for w, i in zip(ws, ids)]

    def GetMappoint(self, point_id: int):
        p = np.zeros(3)
        t, n = C.c_int(), C.c_int()
        capi.check(self._lib.rspl_map_get_mappoint(self._h, point_id, _p(p, C.c_double), C.byref(t), C.byref(n),
                                                   None, None, 0), "rspl_map_get_mappoint")
        fr, kp = np.zeros(n.value, np.int32), np.zeros(n.value, np.int32)
        capi.check(self._lib.rspl_map_get_mappoint(self._h, point_id, None, None, None, _p(fr, C.c_int32),
                                                   _p(kp, C.c_int32), n.value), "rspl_map_get_mappoint")
        return p, t.value, {int(f): int(k) for f, k in zip(fr, kp)}

    def GetMapline(self, line_id: int):
        L, ep = np.zeros(6), np.zeros(6)
        t, n, v = C.c_int(), C.c_int(), C.c_int()
        capi.check(self._lib.rspl_map_get_mapline(self._h, line_id, _p(L, C.c_double), C.byref(t), C.byref(n),
                                                  _p(ep, C.c_double), C.byref(v)), "rspl_map_get_mapline")
        return L, t.value, n.value, ep, bool(v.value)

    def FrameSlots(self, frame_id: int):
        """(Frame::_mappoints, Frame::_maplines) as landmark ids (-1 = nullptr)."""
        a = np.zeros(self._nkp[frame_id], np.int32)
        b = np.zeros(self._nl[frame_id], np.int32)
        capi.check(self._lib.rspl_map_get_frame_slots(self._h, frame_id, _p(a, C.c_int32), _p(b, C.c_int32)),
                   "rspl_map_get_frame_slots")
        return a, b

    def SaveKeyframeTrajectory(self, path: str):
        capi.check(self._lib.rspl_map_save_trajectory(self._h, str(path).encode()), "rspl_map_save_trajectory")
