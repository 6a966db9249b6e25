"""Line front end over the rspl_line* C ABI.

Mirrors the reference's free functions and LineDetector (include/line_processor.h:22-61):

  LineDetector              createFastLineDetector(config) + LineExtractor(image) (line_processor.cc:
                            455-490): cv::resize(0.5) + FLD (restated: GPU resize / Sobel / Canny
                            classification, host hysteresis / chaining / fitting), then the merges
  LineExtractor(segments)   LineDetector::LineExtractor after fld->detect (line_processor.cc:460-490):
                            the x2 scale and the two MergeLines / FilterShortLines passes (host C++)
  AssignPointsToLines       line_processor.cc:163-216 (GPU) -> list of {point index: distance}
  MatchLines                line_processor.cc:221-283 (GPU) -> line_matches (-1 = unmatched)
  StereoLines               the line part of Frame::AddLeftFeatures / AddRightFeatures
                            (frame.cc:124-129, 150-196) in one call
  stereo_lines_device       the same, device-resident (SuperPoint / SuperGlue device outputs in,
                            device right lines out, stream-ordered)

FLD (cv::ximgproc::FastLineDetector, OpenCV contrib, absent) is restated (parity unpinned); the
RCF edge network is not rebuilt (no weights): its edge map is LineDetector's input.  There is no
CPU path for the GPU functions.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Sequence, Tuple

import numpy as np

from . import capi

_i32p, _u8p, _dp, _fp = C.POINTER(C.c_int32), C.POINTER(C.c_uint8), C.POINTER(C.c_double), C.POINTER(C.c_float)


class LinesConfig(C.Structure):
    _fields_ = [("max_lines", C.c_int), ("max_points", C.c_int), ("max_pairs", C.c_int),
                ("max_matches", C.c_int), ("device", C.c_int)]


class FldConfig(C.Structure):
    """rspl_fld_config = LineDetectorConfig's FLD fields (configs/configs_euroc.yaml:31-35)"""
    _fields_ = [("length_threshold", C.c_int), ("distance_threshold", C.c_double), ("canny_th1", C.c_double),
                ("canny_th2", C.c_double), ("canny_aperture_size", C.c_int)]


def _declare(lib):
    if getattr(lib, "_rspl_lines_declared", False):
        return lib
    vp, ip = C.c_void_p, C.c_int
    lib.rspl_line_extract.argtypes = [_fp, ip, ip, _dp, ip, C.POINTER(ip)]
    lib.rspl_lines_create.argtypes = [C.POINTER(LinesConfig), C.POINTER(vp)]
    lib.rspl_lines_destroy.argtypes = [vp]
    lib.rspl_lines_destroy.restype = None
    lib.rspl_lines_assign.argtypes = [vp, _dp, ip, _dp, ip, _i32p, _i32p, _dp, ip]
    lib.rspl_lines_match.argtypes = [vp, _i32p, _i32p, ip, _i32p, _i32p, ip, _i32p, ip, ip, ip, _i32p]
    lib.rspl_lines_stereo.argtypes = [vp, _dp, ip, _dp, ip, _dp, ip, _dp, ip, _i32p, ip, _dp, _dp, _u8p,
                                      C.POINTER(ip)]
    lib.rspl_lines_stereo_device.argtypes = [vp, vp, ip, vp, ip, vp, ip, vp, vp, _dp, vp, vp, vp]
    lib.rspl_lines_status.argtypes = [vp, C.POINTER(ip)]
    lib.rspl_lines_detect.argtypes = [vp, _u8p, ip, ip, ip, C.POINTER(FldConfig), _fp, ip, C.POINTER(ip)]
    lib.rspl_lines_debug_canny.argtypes = [vp, ip, ip, _u8p, _u8p]
    lib.rspl_lines_extract_async.argtypes = [vp, _u8p, ip, ip, ip, C.POINTER(FldConfig), ip]
    lib.rspl_lines_extract_wait.argtypes = [vp, _dp, ip, C.POINTER(ip), _dp]
    lib.rspl_lines_extract_wait_device.argtypes = [vp, vp, ip, C.POINTER(ip), _dp, vp]
    lib._rspl_lines_declared = True
    return lib


def _p(a, ct):
    return a.ctypes.data_as(C.POINTER(ct)) if a is not None and a.size else None


def _features(features: np.ndarray) -> np.ndarray:
    """The reference's Eigen::Matrix<double, 259, Dynamic> (column-major) = [N][259] records."""
    f = np.asarray(features, dtype=np.float64)
    if f.ndim == 2 and f.shape[0] == 259 and f.shape[1] != 259:
        f = f.T
    return np.ascontiguousarray(f.reshape(-1, 259))


def LineExtractor(segments: np.ndarray, do_merge: bool = True) -> np.ndarray:
    """Segments [n][4] (FLD on the half-size image) -> lines [m][4] double at full size."""
    lib = _declare(capi.load())
    s = np.ascontiguousarray(segments, dtype=np.float32).reshape(-1, 4)
    cap = max(1, len(s))
    out = np.zeros((cap, 4), np.float64)
    n = C.c_int()
    capi.check(lib.rspl_line_extract(_p(s, C.c_float), len(s), int(do_merge), _p(out, C.c_double), cap, C.byref(n)),
               "rspl_line_extract")
    return out[: n.value].copy()


def relation_to_csr(relation: Sequence[Dict[int, float]]) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    off = np.zeros(len(relation) + 1, np.int32)
    idx, dist = [], []
    for i, m in enumerate(relation):
        keys = sorted(m)
        idx += keys
        dist += [m[k] for k in keys]
        off[i + 1] = len(idx)
    return off, np.asarray(idx, np.int32), np.asarray(dist, np.float64)


def csr_to_relation(off, idx, dist) -> List[Dict[int, float]]:
    return [{int(idx[e]): float(dist[e]) for e in range(off[i], off[i + 1])} for i in range(len(off) - 1)]


class LineMatcher:
    """GPU handle for AssignPointsToLines / MatchLines (device memory allocated once)."""

    def __init__(self, max_lines=512, max_points=2048, max_pairs=65536, max_matches=4096, device=0):
        self._lib = _declare(capi.load())
        self.cfg = LinesConfig(max_lines, max_points, max_pairs, max_matches, device)
        self._h = C.c_void_p()
        capi.check(self._lib.rspl_lines_create(C.byref(self.cfg), C.byref(self._h)), "rspl_lines_create")

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            self._lib.rspl_lines_destroy(self._h)
            self._h = C.c_void_p()

    def assign_csr(self, lines: np.ndarray, features: np.ndarray):
        L = np.ascontiguousarray(lines, np.float64).reshape(-1, 4)
        F = _features(features)
        off = np.zeros(len(L) + 1, np.int32)
        cap = self.cfg.max_pairs
        idx = np.zeros(cap, np.int32)
        dist = np.zeros(cap, np.float64)
        capi.check(self._lib.rspl_lines_assign(self._h, _p(L, C.c_double), len(L), _p(F, C.c_double), len(F),
                                               off.ctypes.data_as(_i32p), idx.ctypes.data_as(_i32p),
                                               dist.ctypes.data_as(_dp), cap), "rspl_lines_assign")
        n = int(off[-1])
        return off, idx[:n].copy(), dist[:n].copy()

    def AssignPointsToLines(self, lines: np.ndarray, features: np.ndarray) -> List[Dict[int, float]]:
        return csr_to_relation(*self.assign_csr(lines, features))

    def MatchLines(self, points_on_line0, points_on_line1, point_matches, point_num0: int,
                   point_num1: int) -> List[int]:
        """points_on_line*: list of {point: distance} (or CSR triples); point_matches [m][2]."""
        c0 = points_on_line0 if isinstance(points_on_line0, tuple) else relation_to_csr(points_on_line0)
        c1 = points_on_line1 if isinstance(points_on_line1, tuple) else relation_to_csr(points_on_line1)
        m = np.ascontiguousarray(point_matches, np.int32).reshape(-1, 2)
        n0, n1 = len(c0[0]) - 1, len(c1[0]) - 1
        out = np.full(max(1, n0), -1, np.int32)
        o0, i0 = np.ascontiguousarray(c0[0], np.int32), np.ascontiguousarray(c0[1], np.int32)
        o1, i1 = np.ascontiguousarray(c1[0], np.int32), np.ascontiguousarray(c1[1], np.int32)
        capi.check(self._lib.rspl_lines_match(self._h, o0.ctypes.data_as(_i32p), _p(i0, C.c_int32), n0,
                                              o1.ctypes.data_as(_i32p), _p(i1, C.c_int32), n1, _p(m, C.c_int32),
                                              len(m), int(point_num0), int(point_num1), out.ctypes.data_as(_i32p)),
                   "rspl_lines_match")
        return [int(v) for v in out[:n0]]

    def StereoLines(self, lines_left, features_left, lines_right, features_right, stereo_matches,
                    camera_limits: Sequence[float]):
        """-> (lines_right [n_left][4], valid [n_left] bool, kept stereo match count)."""
        Ll = np.ascontiguousarray(lines_left, np.float64).reshape(-1, 4)
        Lr = np.ascontiguousarray(lines_right, np.float64).reshape(-1, 4)
        Fl, Fr = _features(features_left), _features(features_right)
        m = np.ascontiguousarray(stereo_matches, np.int32).reshape(-1, 2)
        lim = np.ascontiguousarray(camera_limits, np.float64)
        out = np.zeros((max(1, len(Ll)), 4), np.float64)
        valid = np.zeros(max(1, len(Ll)), np.uint8)
        kept = C.c_int()
        capi.check(self._lib.rspl_lines_stereo(self._h, _p(Ll, C.c_double), len(Ll), _p(Fl, C.c_double), len(Fl),
                                               _p(Lr, C.c_double), len(Lr), _p(Fr, C.c_double), len(Fr),
                                               _p(m, C.c_int32), len(m), lim.ctypes.data_as(_dp),
                                               out.ctypes.data_as(_dp), valid.ctypes.data_as(_u8p), C.byref(kept)),
                   "rspl_lines_stereo")
        n = len(Ll)
        return out[:n].copy(), valid[:n].astype(bool), kept.value

    def stereo_lines_device(self, d_lines_left: int, n_left: int, d_lines_right: int, n_right: int,
                            d_features: int, feat_cap: int, d_counts: int, d_match_idx: int,
                            camera_limits: Sequence[float], d_lines_right_out: int, d_valid: int, stream=None):
        """rspl_lines_stereo_device on raw device pointers (see include/rspl.h)."""
        lim = np.ascontiguousarray(camera_limits, np.float64)
        capi.check(self._lib.rspl_lines_stereo_device(self._h, d_lines_left, n_left, d_lines_right, n_right,
                                                      d_features, feat_cap, d_counts, d_match_idx,
                                                      lim.ctypes.data_as(_dp), d_lines_right_out, d_valid, stream),
                   "rspl_lines_stereo_device")

    def status(self) -> bool:
        """True when an assignment of the last device call overflowed max_pairs."""
        o = C.c_int()
        capi.check(self._lib.rspl_lines_status(self._h, C.byref(o)), "rspl_lines_status")
        return bool(o.value)


class LineDetector:
    """LineDetector (include/line_processor.h, line_processor.cc:455-490): the FLD of the half-size
    image (rspl_lines_detect) and LineExtractor's scale + merge passes (rspl_line_extract)."""

    def __init__(self, length_threshold=10, distance_threshold=1.414213562, canny_th1=200.0, canny_th2=250.0,
                 canny_aperture_size=3, do_merge=True, max_segments=16384, device=0):
        self._lib = _declare(capi.load())
        self.cfg = FldConfig(length_threshold, distance_threshold, canny_th1, canny_th2, canny_aperture_size)
        self.do_merge = do_merge
        self._seg = np.zeros((max_segments, 4), np.float32)
        self._h = C.c_void_p()
        lc = LinesConfig(1, 1, 1, 0, device)
        capi.check(self._lib.rspl_lines_create(C.byref(lc), C.byref(self._h)), "rspl_lines_create")

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            self._lib.rspl_lines_destroy(self._h)
            self._h = C.c_void_p()

    def detect(self, image: np.ndarray) -> np.ndarray:
        """fld->detect(cv::resize(image, 0.5)): segments [n][4] float32 on the half image"""
        img = np.ascontiguousarray(image, np.uint8)
        n = C.c_int()
        capi.check(self._lib.rspl_lines_detect(self._h, _p(img, C.c_uint8), img.shape[0], img.shape[1], img.shape[1],
                                               C.byref(self.cfg), _p(self._seg, C.c_float), len(self._seg),
                                               C.byref(n)), "rspl_lines_detect")
        return self._seg[: n.value].copy()

    def debug_canny(self, H: int, W: int):
        """the last detect's half image and Canny classes (2 strong, 0 candidate, 1 none)"""
        half = np.zeros((H // 2, W // 2), np.uint8)
        cls = np.zeros_like(half)
        capi.check(self._lib.rspl_lines_debug_canny(self._h, H, W, _p(half, C.c_uint8), _p(cls, C.c_uint8)),
                   "rspl_lines_debug_canny")
        return half, cls

    def LineExtractor(self, image: np.ndarray) -> np.ndarray:
        """lines [m][4] double at full size (x2 scale; the merges when do_merge)"""
        return LineExtractor(self.detect(image), self.do_merge)

    def submit(self, image: np.ndarray):
        """LineExtractor(image) on the handle's native worker thread (rspl_lines_extract_async); the
        image is kept alive until wait() returns its lines"""
        img = np.ascontiguousarray(image, np.uint8)
        self._job_img = img
        capi.check(self._lib.rspl_lines_extract_async(self._h, _p(img, C.c_uint8), img.shape[0], img.shape[1],
                                                      img.shape[1], C.byref(self.cfg), int(self.do_merge)),
                   "rspl_lines_extract_async")

    def wait(self, capacity: int = 4096):
        """the submitted job's lines [m][4] double at full size and the job's duration on the worker in ms
        (rspl_lines_extract_wait)"""
        out = np.zeros((capacity, 4), np.float64)
        n, us = C.c_int(), C.c_double()
        rc = self._lib.rspl_lines_extract_wait(self._h, _p(out, C.c_double), capacity, C.byref(n), C.byref(us))
        self._job_img = None
        capi.check(rc, "rspl_lines_extract_wait")
        return out[: n.value], us.value / 1e3

    def wait_device(self, d_lines: int, capacity: int, stream=None):
        """the submitted job's lines copied to device memory d_lines [capacity][4] in stream order
        (rspl_lines_extract_wait_device); returns (n, job ms)"""
        n, us = C.c_int(), C.c_double()
        rc = self._lib.rspl_lines_extract_wait_device(self._h, d_lines, capacity, C.byref(n), C.byref(us), stream)
        self._job_img = None
        capi.check(rc, "rspl_lines_extract_wait_device")
        return n.value, us.value / 1e3

