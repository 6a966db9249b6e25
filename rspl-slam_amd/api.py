"""Host-side mirror of the reference's C++ classes for the hot path, over the C ABI.

  SuperPoint     include/super_point.h:20-66      (build / infer)
  SuperGlue      include/super_glue.h:20-71       (build / infer)
  PointMatching  include/point_matching.h:7-18    (MatchingPoints / NormalizeKeypoints)
  LocalmapOptimization  include/g2o_optimization/g2o_optimization.h:15-19
  FrameOptimization     include/g2o_optimization/g2o_optimization.h:20-22
  SolvePnPWithCV        include/g2o_optimization/g2o_optimization.h:24

Same names and argument meaning as the reference; C++ out-parameters become
return values ((ok, features) for SuperPoint::infer, etc.).  Everything runs
in librspl.so on the MI355X -- no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

from . import capi


@dataclass
class SuperPointConfig:               # include/read_configs.h:9-18 (+ device arena sizing)
    max_keypoints: int = 400
    keypoint_threshold: float = 0.004
    remove_borders: int = 4
    weights: str = ""                 # RSPLWT01 blob (replaces onnx_file / engine_file)
    max_height: int = 480
    max_width: int = 752
    max_batch: int = 2
    precision: int = capi.RSPL_PREC_FP32
    device: int = 0


class SuperPoint:
    """Mirror of class SuperPoint (include/super_point.h:20-66)."""

    def __init__(self, super_point_config: SuperPointConfig):
        self.config = super_point_config
        self._h = C.c_void_p()
        self._lib = capi.load()

    def build(self) -> bool:
        c = self.config
        cfg = capi.SpConfig(c.max_keypoints, c.keypoint_threshold, c.remove_borders, c.max_height, c.max_width,
                            c.max_batch, c.precision, c.device)
        rc = self._lib.rspl_sp_create(C.byref(cfg), c.weights.encode(), C.byref(self._h))
        self.error = None if rc == 0 else self._lib.rspl_last_error().decode()
        return rc == 0

    def _cap(self):
        return self.config.max_keypoints if self.config.max_keypoints > 0 else 16384

    def infer(self, image: np.ndarray) -> Tuple[bool, np.ndarray]:
        """SuperPoint::infer (src/super_point.cpp:104-135): u8 [H, W] -> (ok, features [259, N])."""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        H, W = img.shape
        cap = self._cap()
        out = np.empty((cap, 259), np.float64)
        n = C.c_int(0)
        rc = self._lib.rspl_sp_infer(self._h, img.ctypes.data, H, W, W, out.ctypes.data, cap, C.byref(n))
        if rc != 0:
            self.error = self._lib.rspl_last_error().decode()
            return False, np.zeros((259, 0))
        return True, np.ascontiguousarray(out[: n.value].T)

    def infer_device(self, d_images: int, batch: int, height: int, width: int, stride: int, pitch: int,
                     d_features: int, capacity: int, d_counts: int, stream: Optional[int] = None) -> None:
        """Batched device-resident form (pointers are device addresses, e.g. torch tensor data_ptr())."""
        capi.check(self._lib.rspl_sp_infer_device(self._h, d_images, batch, height, width, stride, pitch,
                                                  d_features, capacity, d_counts, stream), "rspl_sp_infer_device")

    STAGES = ("conv1a+1b+pool", "conv2a..conv4b", "convPa|convDa", "heads 1x1", "nms", "topk", "sample")

    def profile(self, enable: bool = True):
        capi.check(self._lib.rspl_sp_profile(self._h, int(enable)), "rspl_sp_profile")

    def stage_times(self):
        """(per-stage summed ms, calls) since profile(True)"""
        return capi.stage_times(None, self._lib.rspl_sp_stage_times, self._h, len(self.STAGES))

    def debug_nms(self, scores: np.ndarray) -> np.ndarray:
        """The device simple_nms (superpoint.py:6-33) of a host score map."""
        sc = np.ascontiguousarray(scores, np.float32)
        out = np.empty_like(sc)
        capi.check(self._lib.rspl_sp_debug_nms(self._h, sc.ctypes.data, sc.shape[0], sc.shape[1], out.ctypes.data),
                   "rspl_sp_debug_nms")
        return out

    def debug_maps(self, b: int, height: int, width: int):
        s = np.empty((height, width), np.float32)
        d = np.empty((256, height // 8, width // 8), np.float32)
        capi.check(self._lib.rspl_sp_debug_maps(self._h, b, s.ctypes.data, d.ctypes.data), "rspl_sp_debug_maps")
        return s, d

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            self._lib.rspl_sp_destroy(self._h)
            self._h = C.c_void_p()


@dataclass
class SuperGlueConfig:                # include/read_configs.h:20-28 (+ arena sizing)
    image_width: int = 752
    image_height: int = 480
    weights: str = ""                 # RSPLWT01 blob (replaces onnx_file / engine_file)
    max_keypoints: int = 400
    max_batch: int = 2
    sinkhorn_iterations: int = 100
    precision: int = capi.RSPL_PREC_FP32
    device: int = 0


class SuperGlue:
    """Mirror of class SuperGlue (include/super_glue.h:20-71)."""

    def __init__(self, superglue_config: SuperGlueConfig):
        self.config = superglue_config
        self._h = C.c_void_p()
        self._lib = capi.load()
        self.error = None

    def build(self) -> bool:
        c = self.config
        cfg = capi.SgConfig(c.image_width, c.image_height, c.max_keypoints, c.max_batch, c.sinkhorn_iterations,
                            c.precision, c.device)
        rc = self._lib.rspl_sg_create(C.byref(cfg), c.weights.encode(), C.byref(self._h))
        self.error = None if rc == 0 else self._lib.rspl_last_error().decode()
        return rc == 0

    def infer(self, features0: np.ndarray, features1: np.ndarray):
        """SuperGlue::infer (src/super_glue.cpp:137-197) on NORMALISED 259 x n features.
        Returns (ok, indices0, indices1, mscores0, mscores1)."""
        f0 = np.ascontiguousarray(np.asarray(features0, np.float64).T)
        f1 = np.ascontiguousarray(np.asarray(features1, np.float64).T)
        n0, n1 = f0.shape[0], f1.shape[0]
        i0, i1 = np.empty(n0, np.int32), np.empty(n1, np.int32)
        m0, m1 = np.empty(n0, np.float64), np.empty(n1, np.float64)
        rc = self._lib.rspl_sg_infer(self._h, f0.ctypes.data, n0, f1.ctypes.data, n1, i0.ctypes.data, i1.ctypes.data,
                                     m0.ctypes.data, m1.ctypes.data)
        if rc != 0:
            self.error = self._lib.rspl_last_error().decode()
            return False, i0, i1, m0, m1
        return True, i0, i1, m0, m1

    def infer_device(self, batch: int, d_feat0: int, d_n0: int, d_feat1: int, d_n1: int, stride_feat: int,
                     normalize: bool, d_idx0: int, d_idx1: int, d_ms0: int, d_ms1: int, stream=None,
                     post_stream=None) -> None:
        """Device-resident batched SuperGlue; with post_stream, Sinkhorn + decode run there
        (results complete on post_stream) so the next call's GNN overlaps them."""
        if post_stream is None:
            capi.check(self._lib.rspl_sg_infer_device(self._h, batch, d_feat0, d_n0, d_feat1, d_n1, stride_feat,
                                                      int(normalize), d_idx0, d_idx1, d_ms0, d_ms1, stream),
                       "rspl_sg_infer_device")
        else:
            capi.check(self._lib.rspl_sg_infer_device2(self._h, batch, d_feat0, d_n0, d_feat1, d_n1, stride_feat,
                                                       int(normalize), d_idx0, d_idx1, d_ms0, d_ms1, stream,
                                                       post_stream), "rspl_sg_infer_device2")

    STAGES = ("prep+kenc", "gnn x18", "final+scores", "post hand-over", "sinkhorn", "decode")

    def profile(self, enable: bool = True):
        capi.check(self._lib.rspl_sg_profile(self._h, int(enable)), "rspl_sg_profile")

    def stage_times(self):
        return capi.stage_times(None, self._lib.rspl_sg_stage_times, self._h, len(self.STAGES))

    def debug_scores(self, p: int, n0: int, n1: int) -> np.ndarray:
        Z = np.empty((n0 + 1, n1 + 1), np.float32)
        capi.check(self._lib.rspl_sg_debug_scores(self._h, p, Z.ctypes.data), "rspl_sg_debug_scores")
        return Z

    def status(self):
        """rspl_sg_status: (ok, failed-pair bitmask) of the device paths since the last check
        (call after synchronising the stream the results were produced on)."""
        f = C.c_uint32(0)
        rc = self._lib.rspl_sg_status(self._h, C.byref(f))
        if rc != 0:
            self.error = self._lib.rspl_last_error().decode()
        return rc == 0, f.value

    def debug_inject(self, inject: bool, spin_limit: int = 0):
        capi.check(self._lib.rspl_sg_debug_inject(self._h, int(inject), spin_limit), "rspl_sg_debug_inject")

    def debug_sinkhorn(self, scores: np.ndarray, alpha: float, iters: int = 100):
        """bins + log_optimal_transport (superglue.py:185-205) of a host score matrix on the device.
        Returns (ok, Z)."""
        sc = np.ascontiguousarray(scores, np.float32)
        n0, n1 = sc.shape
        Z = np.empty((n0 + 1, n1 + 1), np.float32)
        rc = self._lib.rspl_sg_debug_sinkhorn(self._h, sc.ctypes.data, n0, n1, float(alpha), iters, Z.ctypes.data)
        if rc != 0:
            self.error = self._lib.rspl_last_error().decode()
        return rc == 0, Z

    def debug_decode(self, Z: np.ndarray):
        """The device decode (src/super_glue.cpp:258-367) of a host log-assignment matrix."""
        z = np.ascontiguousarray(Z, np.float32)
        n0, n1 = z.shape[0] - 1, z.shape[1] - 1
        i0, i1 = np.empty(n0, np.int32), np.empty(n1, np.int32)
        m0, m1 = np.empty(n0, np.float64), np.empty(n1, np.float64)
        capi.check(self._lib.rspl_sg_debug_decode(self._h, z.ctypes.data, n0, n1, i0.ctypes.data, i1.ctypes.data,
                                                  m0.ctypes.data, m1.ctypes.data), "rspl_sg_debug_decode")
        return i0, i1, m0, m1

    @property
    def handle(self):
        return self._h

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            self._lib.rspl_sg_destroy(self._h)
            self._h = C.c_void_p()


class PointMatching:
    """Mirror of class PointMatching (include/point_matching.h:7-18, src/point_matching.cc)."""

    def __init__(self, superglue_config: SuperGlueConfig):
        self._superglue_config = superglue_config
        self.superglue = SuperGlue(superglue_config)
        if not self.superglue.build():
            print("Erron in superglue building")   # src/point_matching.cc:8 (message kept verbatim)

    def MatchingPoints(self, features0: np.ndarray, features1: np.ndarray, outlier_rejection: bool = False):
        """Returns (num_matches, [(queryIdx, trainIdx, distance)])."""
        f0 = np.ascontiguousarray(np.asarray(features0, np.float64).T)
        f1 = np.ascontiguousarray(np.asarray(features1, np.float64).T)
        cap = max(1, min(f0.shape[0], f1.shape[0]))
        out = (capi.DMatch * cap)()
        n = C.c_int(0)
        capi.check(self.superglue._lib.rspl_pm_match(self.superglue.handle, f0.ctypes.data, f0.shape[0],
                                                     f1.ctypes.data, f1.shape[0], out, cap, C.byref(n),
                                                     int(outlier_rejection)), "rspl_pm_match")
        matches = [(out[i].query_idx, out[i].train_idx, out[i].distance) for i in range(n.value)]
        return n.value, matches

    @staticmethod
    def NormalizeKeypoints(features: np.ndarray, width: int, height: int) -> np.ndarray:
        """src/point_matching.cc:50-62 (host helper; the device path normalises in-kernel)."""
        g = np.array(features, np.float64, copy=True)
        scale = max(width, height) * 0.7
        g[1] = (features[1] - width // 2) / scale
        g[2] = (features[2] - height // 2) / scale
        return g


# ---------------------------------------------------------------------------
# Local BA: LocalmapOptimization (include/g2o_optimization/g2o_optimization.h:15-19)
# ---------------------------------------------------------------------------
class LocalBA:
    """Owns one rspl_ba handle (device arena sized once) and runs dense problems."""

    def __init__(self, max_poses=32, max_points=20000, max_lines=2000, max_edges=200000, device=0):
        self._lib = capi.load()
        self._h = C.c_void_p()
        cfg = capi.BaConfig(max_poses, max_points, max_lines, max_edges, device)
        capi.check(self._lib.rspl_ba_create(C.byref(cfg), C.byref(self._h)), "rspl_ba_create")

    def run(self, problem, out=None):
        """problem: ba_types.DenseProblem -> ba_types.DenseResult.  out: a DenseResult of a problem with
        the same shapes to write into (no per-call allocation; its previous contents are overwritten)."""
        from .ba_types import DenseResult
        res = out if out is not None and out.fits(problem) else DenseResult.alloc(problem)
        P, R = problem.to_ctypes(), res.to_ctypes()
        capi.check(self._lib.rspl_ba_local(self._h, C.byref(P), C.byref(R)), "rspl_ba_local")
        res.read_back(R)
        return res

    def submit(self, problem, out=None):
        """Queue `problem` for the handle's native tracking thread (rspl_ba_submit: runs the queued calls
        in order; blocks while two are waiting, as the reference's feature thread).  Returns the result
        buffer the call will write (read it after join()); problem and out are kept alive until then."""
        from .ba_types import DenseResult
        res = out if out is not None and out.fits(problem) else DenseResult.alloc(problem)
        P, R = problem.to_ctypes(), res.to_ctypes()
        inflight = self.__dict__.setdefault("_inflight", [])
        inflight.append((problem, res, P, R))
        capi.check(self._lib.rspl_ba_submit(self._h, C.byref(P), C.byref(R)), "rspl_ba_submit")
        return res

    def join(self):
        """Wait for every submitted call (rspl_ba_join); raises on the first failure.  Returns
        (calls, LM iterations summed over them, their summed wall time in ms) since the last join."""
        n, it, ms = C.c_longlong(), C.c_longlong(), C.c_double()
        rc = self._lib.rspl_ba_join(self._h, C.byref(n), C.byref(it), C.byref(ms))
        inflight, self._inflight = self.__dict__.get("_inflight", []), []
        for _, res, _, R in inflight:
            res.read_back(R)
        capi.check(rc, "rspl_ba_join")
        return n.value, it.value, ms.value

    def kernel_timing(self, every: int):
        """HIP-event timing of the LM trials' two launches on every `every`-th call (0: off)."""
        capi.check(self._lib.rspl_ba_kernel_timing(self._h, every), "rspl_ba_kernel_timing")

    def kernel_times(self):
        """{"chunks+solve": (total ms, launches), "update": (total ms, launches)} since the last read."""
        ms, n = (C.c_double * 2)(), (C.c_longlong * 2)()
        capi.check(self._lib.rspl_ba_kernel_times(self._h, ms, n), "rspl_ba_kernel_times")
        return {"chunks+solve": (ms[0], n[0]), "update": (ms[1], n[1])}

    def set_line_jacobian(self, analytic: bool):
        """Line edges' Jacobians: g2o's central difference (False, the default) or its analytic limit (True)."""
        capi.check(self._lib.rspl_ba_set_line_jacobian(self._h, 1 if analytic else 0), "rspl_ba_set_line_jacobian")

    def trace(self, cap=4096):
        """The host timeline of the calls since the last read (rspl_ba_trace): a list of dicts with
        capi.BA_TRACE_FIELDS (times in time.perf_counter seconds); [] with a library that lacks it."""
        if not hasattr(self._lib, "rspl_ba_trace"):
            return []
        buf, n = (C.c_double * (cap * capi.BA_TRACE_W))(), C.c_int()
        capi.check(self._lib.rspl_ba_trace(self._h, buf, cap, C.byref(n)), "rspl_ba_trace")
        a = np.frombuffer(buf, np.float64, n.value * capi.BA_TRACE_W).reshape(n.value, capi.BA_TRACE_W)
        return [dict(zip(capi.BA_TRACE_FIELDS, map(float, row))) for row in a]

    def use_reserved_cus(self, reserve_cus: int):
        """Confine this handle's kernels to the CUs reserving streams leave free (0 = all CUs)."""
        capi.check(self._lib.rspl_ba_use_reserved_cus(self._h, reserve_cus), "rspl_ba_use_reserved_cus")

    def set_group(self, group: "ShardGroup", rank: int):
        """Landmark-sharded solve: this handle is rank `rank` of an in-process group (one device)."""
        capi.check(self._lib.rspl_ba_set_group(self._h, group.handle, rank), "rspl_ba_set_group")
        self._shard = group  # keep the group alive while the handle uses it

    def set_shard(self, rank: int, nranks: int, host_allreduce):
        """Landmark-sharded solve over any host transport: host_allreduce(x) sums the float64 numpy
        array x in place across the ranks (e.g. a gloo / MPI all-reduce).  The device buffer of each
        per-trial all-reduce is staged through host memory (rspl_allreduce_fn, stream-ordered)."""
        lib = self._lib
        AR = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)

        def cb(ctx, d_buf, count, stream):
            try:
                h = np.empty(count, np.float64)
                if lib.rspl_memcpy_d2h(h.ctypes.data, d_buf, count * 8, stream):
                    return -1
                host_allreduce(h)
                return 1 if lib.rspl_memcpy_h2d(d_buf, h.ctypes.data, count * 8, stream) else 0
            except Exception:  # the C side turns a non-zero return into RSPL_E_DEVICE
                return -1
        self._ar_cb = AR(cb)  # keep the trampoline alive as long as the handle
        capi.check(lib.rspl_ba_set_shard(self._h, rank, nranks, self._ar_cb, None), "rspl_ba_set_shard")

    def set_comm(self, comm: "Comm"):
        """Landmark-sharded solve across processes / GPUs over RCCL (one rank per GPU)."""
        capi.check(self._lib.rspl_ba_set_comm(self._h, comm.handle), "rspl_ba_set_comm")
        self._shard = comm

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            self._lib.rspl_ba_destroy(self._h)
            self._h = C.c_void_p()


class ShardGroup:
    """rspl_group: nranks LocalBA handles on one device, each driven by its own host thread."""

    def __init__(self, nranks: int):
        self._lib = capi.load()
        self.handle = C.c_void_p()
        self.nranks = nranks
        capi.check(self._lib.rspl_group_create(nranks, C.byref(self.handle)), "rspl_group_create")

    def __del__(self):
        if getattr(self, "handle", None) and self.handle.value:
            self._lib.rspl_group_destroy(self.handle)
            self.handle = C.c_void_p()


COMM_ID_BYTES = 128


def comm_unique_id() -> bytes:
    """RCCL unique id (rank 0 makes it; broadcast it out of band, e.g. with torch.distributed)."""
    buf = (C.c_uint8 * COMM_ID_BYTES)()
    capi.check(capi.load().rspl_comm_unique_id(buf), "rspl_comm_unique_id")
    return bytes(buf)


class Comm:
    """rspl_comm: an RCCL communicator (one rank per GPU, xGMI within the node)."""

    def __init__(self, unique_id: bytes, rank: int, nranks: int, device: int = 0):
        self._lib = capi.load()
        self.handle = C.c_void_p()
        self.rank, self.nranks = rank, nranks
        uid = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(unique_id)
        capi.check(self._lib.rspl_comm_create(uid, rank, nranks, device, C.byref(self.handle)), "rspl_comm_create")

    def __del__(self):
        if getattr(self, "handle", None) and self.handle.value:
            self._lib.rspl_comm_destroy(self.handle)
            self.handle = C.c_void_p()


def broadcast_comm_id(group, make_id=comm_unique_id) -> bytes:
    """Rank 0 makes the RCCL id, every rank of the host group (hostgroup.HostGroup) receives it."""
    return group.broadcast_bytes(make_id() if group.rank == 0 else b"")


_default_ba = None


def LocalmapOptimization(poses, points, lines, camera_list, mono_point_constraints, stereo_point_constraints,
                         mono_line_constraints, stereo_line_constraints, cfg) -> None:
    """Same signature and in-place semantics as the reference (g2o_optimization.cc:21-252):
    poses / points / lines (dict id -> Pose3d / Position3d / Line3d) are updated, constraint
    ``inlier`` flags are written."""
    from . import ba_types as BT
    global _default_ba
    dp, ids = BT.pack_problem(poses, points, lines, camera_list, mono_point_constraints, stereo_point_constraints,
                              mono_line_constraints, stereo_line_constraints, cfg)
    need = (len(poses), len(points), len(lines),
            max(len(mono_point_constraints), len(stereo_point_constraints), len(mono_line_constraints),
                len(stereo_line_constraints)))
    if _default_ba is None or any(n > c for n, c in zip(need, _default_ba_caps)):
        caps = tuple(max(n, c) for n, c in zip(need, (32, 20000, 2000, 200000)))
        _default_ba = LocalBA(*caps)
        globals()["_default_ba_caps"] = caps
    res = _default_ba.run(dp)
    BT.unpack_result(res, ids, poses, points, lines, mono_point_constraints, stereo_point_constraints,
                     mono_line_constraints, stereo_line_constraints)


_default_ba_caps = (0, 0, 0, 0)


# ---------------------------------------------------------------------------
# Tracking pose optimisation: FrameOptimization (include/g2o_optimization/g2o_optimization.h:20-22)
# ---------------------------------------------------------------------------
class FrameBA:
    """Owns one rspl_frame handle; optimises a batch of independent frames in one launch."""

    def __init__(self, max_batch=64, max_edges=65536, max_points=65536, device=0):
        self._lib = capi.load()
        self._h = C.c_void_p()
        cfg = capi.FrameConfig(max_batch, max_edges, max_points, device)
        capi.check(self._lib.rspl_frame_create(C.byref(cfg), C.byref(self._h)), "rspl_frame_create")

    def run(self, problems):
        """problems: list of ba_types.FrameProblem -> list of ba_types.FrameResult"""
        from .ba_types import FrameResult, RsplFrameProblem, RsplFrameResult
        res = [FrameResult.alloc(p) for p in problems]
        P = (RsplFrameProblem * len(problems))(*[p.to_ctypes() for p in problems])
        R = (RsplFrameResult * len(problems))(*[r.to_ctypes() for r in res])
        capi.check(self._lib.rspl_frame_optimize(self._h, P, len(problems), R), "rspl_frame_optimize")
        for r, rc in zip(res, R):
            r.read_back(rc)
        return res

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            self._lib.rspl_frame_destroy(self._h)
            self._h = C.c_void_p()


_default_frame = None


def FrameOptimization(poses, points, camera_list, mono_point_constraints, stereo_point_constraints, cfg) -> int:
    """Same signature, in-place semantics and return value as the reference
    (g2o_optimization.cc:256-398): the single pose in ``poses`` is updated, constraint ``inlier``
    flags are written, and the number of inlier constraints is returned."""
    from . import ba_types as BT
    global _default_frame
    fp = BT.pack_frame_problem(poses, points, camera_list, mono_point_constraints, stereo_point_constraints, cfg)
    ne = len(mono_point_constraints) + len(stereo_point_constraints)
    if _default_frame is None or ne > _default_frame_cap[0] or len(points) > _default_frame_cap[1]:
        cap = (max(ne, 65536), max(len(points), 65536))
        _default_frame = FrameBA(max_batch=1, max_edges=cap[0], max_points=cap[1])
        globals()["_default_frame_cap"] = cap
    r = _default_frame.run([fp])[0]
    pose = next(iter(poses.values()))
    pose.q = r.pose_q.copy()
    pose.p = r.pose_p.copy()
    for c, f in zip(mono_point_constraints, r.inlier["mono"]):
        c.inlier = bool(f)
    for c, f in zip(stereo_point_constraints, r.inlier["stereo"]):
        c.inlier = bool(f)
    return r.n_inliers


_default_frame_cap = (0, 0)


# ---------------------------------------------------------------------------
# SolvePnPWithCV (include/g2o_optimization/g2o_optimization.h:24, g2o_optimization.cc:402-461)
# ---------------------------------------------------------------------------
class PnP:
    """Owns one rspl_pnp handle: cv::solvePnPRansac's RANSAC (5-point EPnP hypotheses side by
    side) + refinement, for a batch of frames in one launch."""

    def __init__(self, max_batch=64, max_points=65536, device=0):
        self._lib = capi.load()
        self._h = C.c_void_p()
        cfg = capi.PnpConfig(max_batch, max_points, device)
        capi.check(self._lib.rspl_pnp_create(C.byref(cfg), C.byref(self._h)), "rspl_pnp_create")

    def solve(self, frames, iterations=100, reprojection_error=20.0, confidence=0.99):
        """frames: list of (K4 = (fx, fy, cx, cy), points [n, 3], keypoints [n, 2]).
        Returns a list of (n_inliers, Rwc [3, 3], twc [3], inlier mask [n] uint8, hypotheses)."""
        keep, P, R = [], [], []
        for K4, pts, kps in frames:
            p3 = np.ascontiguousarray(pts, np.float64).reshape(-1, 3)
            p2 = np.ascontiguousarray(kps, np.float64).reshape(-1, 2)
            inl = np.zeros(max(p3.shape[0], 1), np.uint8)
            keep.append((p3, p2, inl))
            P.append(capi.PnpProblem(K4[0], K4[1], K4[2], K4[3], p3.shape[0],
                                     p3.ctypes.data_as(C.POINTER(C.c_double)),
                                     p2.ctypes.data_as(C.POINTER(C.c_double)), iterations, reprojection_error,
                                     confidence))
            r = capi.PnpResult()
            r.inlier = inl.ctypes.data_as(C.POINTER(C.c_uint8))
            R.append(r)
        Pa = (capi.PnpProblem * len(P))(*P)
        Ra = (capi.PnpResult * len(R))(*R)
        capi.check(self._lib.rspl_pnp_solve(self._h, Pa, len(P), Ra), "rspl_pnp_solve")
        return [(r.n_inliers, np.array(r.Rwc[:]).reshape(3, 3), np.array(r.twc[:]), k[2][:k[0].shape[0]].copy(),
                 r.hypotheses) for r, k in zip(Ra, keep)]

    def debug_hypotheses(self, frame=0, max_hyps=128):
        """every hypothesis of frame `frame` of the last solve: (counts int32 [k], -1 = the
        minimal solver failed; poses [k, 12] = R row-major | t)"""
        cnt = np.zeros(max_hyps, np.int32)
        poses = np.zeros((max_hyps, 12))
        k = self._lib.rspl_pnp_debug_hypotheses(self._h, frame, max_hyps, cnt.ctypes.data_as(C.c_void_p),
                                                poses.ctypes.data_as(C.c_void_p))
        if k < 0:
            capi.check(k, "rspl_pnp_debug_hypotheses")
        return cnt[:k], poses[:k]

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            self._lib.rspl_pnp_destroy(self._h)
            self._h = C.c_void_p()


_default_pnp = None


def SolvePnPWithCV(K4, points, keypoints, point_ids=None):
    """The reference's SolvePnPWithCV over already-filtered correspondences (:417-431): returns
    (n_inliers, pose Twc 4x4, inliers) where inliers[i] = point_ids[i] for RANSAC inliers, else -1
    (:452-457; point_ids defaults to the correspondence index)."""
    global _default_pnp
    n = len(points)
    if _default_pnp is None or n > _default_pnp_cap[0]:
        cap = max(n, 65536)
        _default_pnp = PnP(max_batch=1, max_points=cap)
        globals()["_default_pnp_cap"] = (cap,)
    k, Rwc, twc, inl, _ = _default_pnp.solve([(K4, points, keypoints)])[0]
    T = np.eye(4)
    if k > 0:
        T[:3, :3] = Rwc
        T[:3, 3] = twc
    ids = np.arange(n) if point_ids is None else np.asarray(point_ids)
    return k, T, np.where(inl.astype(bool), ids, -1)


_default_pnp_cap = (0,)
