"""ctypes binding of librspl.so (the C ABI declared in include/rspl.h).

This is the product path: every call goes to the HIP library.  There is no CPU
fallback -- if librspl.so is missing or no HIP device is visible, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

PKG = pathlib.Path(__file__).resolve().parent
# RSPL_LIB: another in-tree build of the same ABI (A/B timing of two builds in one GPU call)
LIB_PATH = PKG / os.environ.get("RSPL_LIB", "librspl.so")

RSPL_OK = 0
RSPL_ABI_VERSION = 2  # include/rspl.h: the struct layouts the ctypes mirrors below follow
RSPL_PREC_FP32 = 0
RSPL_PREC_FP16 = 1
RSPL_PREC_FP16X3 = 2  # SuperPoint only: split fp16 (hi + lo planes, three fp16 MFMA products per step)

BA_TRACE_W = 12  # RSPL_BA_TRACE_W
BA_TRACE_FIELDS = ("submit", "stage0", "stage1", "run0", "upload", "opt1", "opt2", "end", "slot", "grew", "iters",  # grew: rspl_ba_trace [9] flags
                   "sync")

EXPORTS = [
    "rspl_last_error", "rspl_version", "rspl_abi_version",
    "rspl_device_count", "rspl_set_device", "rspl_malloc", "rspl_free", "rspl_memcpy_h2d", "rspl_memcpy_d2h",
    "rspl_memset", "rspl_memcpy_d2d", "rspl_stream_create", "rspl_stream_create_priority", "rspl_stream_create_reserving", "rspl_stream_destroy", "rspl_stream_synchronize",
    "rspl_device_synchronize", "rspl_event_create", "rspl_event_record", "rspl_stream_wait_event",
    "rspl_event_destroy", "rspl_timer_create", "rspl_timer_record", "rspl_timer_elapsed_ms",
    "rspl_timer_destroy",
    "rspl_sp_create", "rspl_sp_infer", "rspl_sp_infer_device", "rspl_sp_debug_maps", "rspl_sp_debug_nms", "rspl_sp_profile",
    "rspl_sp_stage_times", "rspl_sp_destroy",
    "rspl_sg_create", "rspl_sg_infer", "rspl_sg_infer_device", "rspl_sg_infer_device2", "rspl_sg_debug_scores", "rspl_sg_profile",
    "rspl_sg_status", "rspl_sg_debug_inject", "rspl_sg_debug_sinkhorn", "rspl_sg_debug_decode",
    "rspl_sg_stage_times", "rspl_sg_destroy",
    "rspl_pm_match",
    "rspl_ba_create", "rspl_ba_local", "rspl_ba_submit", "rspl_ba_join", "rspl_ba_destroy", "rspl_ba_use_reserved_cus", "rspl_ba_kernel_timing",
    "rspl_ba_kernel_times", "rspl_ba_trace", "rspl_ba_set_line_jacobian", "rspl_ba_debug_stage",
    "rspl_frame_create", "rspl_frame_optimize", "rspl_frame_destroy",
    "rspl_ba_set_shard", "rspl_comm_unique_id", "rspl_comm_create", "rspl_comm_allreduce_sum", "rspl_comm_destroy",
    "rspl_ba_set_comm", "rspl_group_create", "rspl_group_destroy", "rspl_ba_set_group",
    "rspl_pnp_create", "rspl_pnp_solve", "rspl_pnp_destroy", "rspl_pnp_debug_hypotheses",
    "rspl_line_extract", "rspl_lines_create", "rspl_lines_destroy", "rspl_lines_assign", "rspl_lines_match",
    "rspl_lines_stereo", "rspl_lines_stereo_device", "rspl_lines_status", "rspl_lines_detect",
    "rspl_lines_debug_canny",
]


class SpConfig(C.Structure):
    _fields_ = [("max_keypoints", C.c_int), ("keypoint_threshold", C.c_double), ("remove_borders", C.c_int),
                ("max_height", C.c_int), ("max_width", C.c_int), ("max_batch", C.c_int),
                ("precision", C.c_int), ("device", C.c_int)]


class SgConfig(C.Structure):
    _fields_ = [("image_width", C.c_int), ("image_height", C.c_int), ("max_keypoints", C.c_int),
                ("max_batch", C.c_int), ("sinkhorn_iterations", C.c_int), ("precision", C.c_int),
                ("device", C.c_int)]


class DMatch(C.Structure):
    _fields_ = [("query_idx", C.c_int32), ("train_idx", C.c_int32), ("distance", C.c_float)]


class BaConfig(C.Structure):
    _fields_ = [("max_poses", C.c_int), ("max_points", C.c_int), ("max_lines", C.c_int),
                ("max_edges", C.c_int), ("device", C.c_int)]


class FrameConfig(C.Structure):
    _fields_ = [("max_batch", C.c_int), ("max_edges", C.c_int), ("max_points", C.c_int), ("device", C.c_int)]


class PnpConfig(C.Structure):
    _fields_ = [("max_batch", C.c_int), ("max_points", C.c_int), ("device", C.c_int)]


class PnpProblem(C.Structure):
    _fields_ = [("fx", C.c_double), ("fy", C.c_double), ("cx", C.c_double), ("cy", C.c_double), ("n", C.c_int),
                ("points", C.POINTER(C.c_double)), ("keypoints", C.POINTER(C.c_double)),
                ("iterations", C.c_int), ("reprojection_error", C.c_double), ("confidence", C.c_double)]


class PnpResult(C.Structure):
    _fields_ = [("Rwc", C.c_double * 9), ("twc", C.c_double * 3), ("inlier", C.POINTER(C.c_uint8)),
                ("n_inliers", C.c_int), ("hypotheses", C.c_int)]


class RsplError(RuntimeError):
    pass


_lib = None


def load(path: pathlib.Path = LIB_PATH):
    """Load librspl.so and declare the C ABI.  Raises if the library is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not path.exists():
        raise RsplError(f"{path} not built: run __graft_entry__.build() (no CPU fallback exists)")
    lib = C.CDLL(str(path))
    vp, ip, dp = C.c_void_p, C.c_int, C.c_double
    lib.rspl_last_error.restype = C.c_char_p
    lib.rspl_version.restype = C.c_char_p
    if lib.rspl_abi_version() != RSPL_ABI_VERSION:
        raise RsplError(f"{path}: ABI {lib.rspl_abi_version()}, these bindings follow ABI {RSPL_ABI_VERSION}: rebuild")
    lib.rspl_sp_create.argtypes = [C.POINTER(SpConfig), C.c_char_p, C.POINTER(vp)]
    lib.rspl_sp_infer.argtypes = [vp, vp, ip, ip, ip, vp, ip, C.POINTER(ip)]
    lib.rspl_sp_infer_device.argtypes = [vp, vp, ip, ip, ip, ip, C.c_size_t, vp, ip, vp, vp]
    lib.rspl_sp_debug_maps.argtypes = [vp, ip, vp, vp]
    lib.rspl_sp_debug_nms.argtypes = [vp, vp, ip, ip, vp]
    lib.rspl_sp_destroy.argtypes = [vp]
    lib.rspl_sp_destroy.restype = None
    lib.rspl_device_count.argtypes = [C.POINTER(ip)]
    lib.rspl_set_device.argtypes = [ip]
    lib.rspl_malloc.argtypes = [C.POINTER(vp), C.c_size_t]
    lib.rspl_free.argtypes = [vp]
    lib.rspl_memcpy_h2d.argtypes = [vp, vp, C.c_size_t, vp]
    lib.rspl_memcpy_d2h.argtypes = [vp, vp, C.c_size_t, vp]
    lib.rspl_memset.argtypes = [vp, ip, C.c_size_t, vp]
    lib.rspl_memcpy_d2d.argtypes = [vp, vp, C.c_size_t, vp]
    lib.rspl_sp_profile.argtypes = [vp, ip]
    lib.rspl_sp_stage_times.argtypes = [vp, C.POINTER(C.c_float), C.POINTER(ip)]
    lib.rspl_stream_create.argtypes = [C.POINTER(vp)]
    lib.rspl_stream_create_priority.argtypes = [C.POINTER(vp), ip]
    lib.rspl_stream_create_reserving.argtypes = [C.POINTER(vp), ip]
    lib.rspl_stream_destroy.argtypes = [vp]
    lib.rspl_stream_synchronize.argtypes = [vp]
    lib.rspl_event_create.argtypes = [C.POINTER(vp)]
    lib.rspl_event_record.argtypes = [vp, vp]
    lib.rspl_stream_wait_event.argtypes = [vp, vp]
    lib.rspl_event_destroy.argtypes = [vp]
    lib.rspl_timer_create.argtypes = [C.POINTER(vp)]
    lib.rspl_timer_record.argtypes = [vp, ip, vp]
    lib.rspl_timer_elapsed_ms.argtypes = [vp, C.POINTER(C.c_float)]
    lib.rspl_timer_destroy.argtypes = [vp]
    lib.rspl_timer_destroy.restype = None
    if hasattr(lib, "rspl_sg_create"):
        lib.rspl_sg_create.argtypes = [C.POINTER(SgConfig), C.c_char_p, C.POINTER(vp)]
        lib.rspl_sg_infer.argtypes = [vp, vp, ip, vp, ip, vp, vp, vp, vp]
        lib.rspl_sg_infer_device.argtypes = [vp, ip, vp, vp, vp, vp, ip, ip, vp, vp, vp, vp, vp]
        lib.rspl_sg_infer_device2.argtypes = [vp, ip, vp, vp, vp, vp, ip, ip, vp, vp, vp, vp, vp, vp]
        lib.rspl_sg_debug_scores.argtypes = [vp, ip, vp]
        lib.rspl_sg_status.argtypes = [vp, C.POINTER(C.c_uint32)]
        lib.rspl_sg_debug_inject.argtypes = [vp, ip, C.c_uint]
        lib.rspl_sg_debug_sinkhorn.argtypes = [vp, vp, ip, ip, C.c_float, ip, vp]
        lib.rspl_sg_debug_decode.argtypes = [vp, vp, ip, ip, vp, vp, vp, vp]
        lib.rspl_sg_profile.argtypes = [vp, ip]
        lib.rspl_sg_stage_times.argtypes = [vp, C.POINTER(C.c_float), C.POINTER(ip)]
        lib.rspl_sg_destroy.argtypes = [vp]
        lib.rspl_sg_destroy.restype = None
        lib.rspl_pm_match.argtypes = [vp, vp, ip, vp, ip, C.POINTER(DMatch), ip, C.POINTER(ip), ip]
    if hasattr(lib, "rspl_ba_create"):
        lib.rspl_ba_create.argtypes = [C.POINTER(BaConfig), C.POINTER(vp)]
        lib.rspl_ba_local.argtypes = [vp, vp, vp]
        lib.rspl_ba_submit.argtypes = [vp, vp, vp]
        lib.rspl_ba_join.argtypes = [vp, vp, vp, vp]
        lib.rspl_ba_use_reserved_cus.argtypes = [vp, ip]
        lib.rspl_ba_kernel_timing.argtypes = [vp, ip]
        lib.rspl_ba_kernel_times.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_longlong)]
        lib.rspl_ba_destroy.argtypes = [vp]
        lib.rspl_ba_destroy.restype = None
        lib.rspl_ba_debug_stage.argtypes = [vp, ip, ip, ip] + [vp] * 9
    if hasattr(lib, "rspl_ba_trace"):  # (absent from older builds used as A/B baselines)
        lib.rspl_ba_trace.argtypes = [vp, C.POINTER(C.c_double), ip, C.POINTER(ip)]
        lib.rspl_ba_set_line_jacobian.argtypes = [vp, ip]
    if hasattr(lib, "rspl_ba_set_shard"):
        lib.rspl_ba_set_shard.argtypes = [vp, ip, ip, vp, vp]
        lib.rspl_comm_unique_id.argtypes = [vp]
        lib.rspl_comm_create.argtypes = [vp, ip, ip, ip, C.POINTER(vp)]
        lib.rspl_comm_allreduce_sum.argtypes = [vp, vp, C.c_size_t, vp]
        lib.rspl_comm_destroy.argtypes = [vp]
        lib.rspl_comm_destroy.restype = None
        lib.rspl_ba_set_comm.argtypes = [vp, vp]
        lib.rspl_group_create.argtypes = [ip, C.POINTER(vp)]
        lib.rspl_group_destroy.argtypes = [vp]
        lib.rspl_group_destroy.restype = None
        lib.rspl_ba_set_group.argtypes = [vp, vp, ip]
    if hasattr(lib, "rspl_pnp_create"):
        lib.rspl_pnp_create.argtypes = [C.POINTER(PnpConfig), C.POINTER(vp)]
        lib.rspl_pnp_solve.argtypes = [vp, vp, ip, vp]
        lib.rspl_pnp_destroy.argtypes = [vp]
        lib.rspl_pnp_destroy.restype = None
        lib.rspl_pnp_debug_hypotheses.argtypes = [vp, C.c_int, C.c_int, vp, vp]
    if hasattr(lib, "rspl_frame_create"):
        lib.rspl_frame_create.argtypes = [C.POINTER(FrameConfig), C.POINTER(vp)]
        lib.rspl_frame_optimize.argtypes = [vp, vp, ip, vp]
        lib.rspl_frame_destroy.argtypes = [vp]
        lib.rspl_frame_destroy.restype = None
    _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != RSPL_OK:
        msg = load().rspl_last_error().decode(errors="replace")
        raise RsplError(f"{what} failed (rc={rc}): {msg}")


# ---------------------------------------------------------------------------
# Device memory / stream / timer wrappers over librspl's own (system ROCm) HIP
# runtime.  Python code in this repo uses these instead of torch.cuda, so only
# one HIP runtime ever drives the device from a process.
# ---------------------------------------------------------------------------
import numpy as _np


class DeviceBuffer:
    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        self._p = C.c_void_p()
        check(load().rspl_malloc(C.byref(self._p), self.nbytes), "rspl_malloc")

    @property
    def ptr(self) -> int:
        return self._p.value

    def offset(self, nbytes: int) -> int:
        return self._p.value + int(nbytes)

    def upload(self, arr: _np.ndarray, stream=None, offset: int = 0):
        a = _np.ascontiguousarray(arr)
        assert offset + a.nbytes <= self.nbytes
        check(load().rspl_memcpy_h2d(self._p.value + offset, a.ctypes.data, a.nbytes, stream), "rspl_memcpy_h2d")
        return self

    def download(self, shape, dtype, stream=None, offset: int = 0) -> _np.ndarray:
        out = _np.empty(shape, dtype)
        assert offset + out.nbytes <= self.nbytes
        check(load().rspl_memcpy_d2h(out.ctypes.data, self._p.value + offset, out.nbytes, stream), "rspl_memcpy_d2h")
        return out

    def zero(self, stream=None):
        check(load().rspl_memset(self._p.value, 0, self.nbytes, stream), "rspl_memset")

    def __del__(self):
        if self._p.value:
            load().rspl_free(self._p)
            self._p = C.c_void_p()


def memcpy_d2d(dst: int, src: int, nbytes: int, stream=None):
    check(load().rspl_memcpy_d2d(dst, src, nbytes, stream), "rspl_memcpy_d2d")


def stage_times(fn_profile, fn_times, handle, nstages):
    ms = (C.c_float * nstages)()
    calls = C.c_int(0)
    check(fn_times(handle, ms, C.byref(calls)), "stage_times")
    return [ms[i] for i in range(nstages)], calls.value


class Event:
    """hipEvent (timing disabled) for cross-stream ordering."""

    def __init__(self):
        self._e = C.c_void_p()
        check(load().rspl_event_create(C.byref(self._e)), "rspl_event_create")

    def record(self, stream):
        check(load().rspl_event_record(self._e, C.c_void_p(stream)), "rspl_event_record")

    def wait_on(self, stream):
        """make `stream` wait for this event"""
        check(load().rspl_stream_wait_event(C.c_void_p(stream), self._e), "rspl_stream_wait_event")

    def __del__(self):
        if self._e.value:
            load().rspl_event_destroy(self._e)
            self._e = C.c_void_p()


class Stream:
    def __init__(self, high_priority: bool = False, reserve_cus: int = 0, priority: str = ""):
        """priority: "" (from high_priority), "high", "normal" or "low" (HIP stream priorities)."""
        self._s = C.c_void_p()
        if not priority:
            priority = "high" if high_priority else "normal"
        if reserve_cus > 0:  # CU-masked: leaves reserve_cus CUs to other (latency-bound) streams
            check(load().rspl_stream_create_reserving(C.byref(self._s), reserve_cus), "rspl_stream_create_reserving")
        elif priority in ("high", "low"):
            check(load().rspl_stream_create_priority(C.byref(self._s), 1 if priority == "high" else 0),
                  "rspl_stream_create_priority")
        else:
            check(load().rspl_stream_create(C.byref(self._s)), "rspl_stream_create")

    @property
    def handle(self) -> int:
        return self._s.value

    def synchronize(self):
        check(load().rspl_stream_synchronize(self._s), "rspl_stream_synchronize")

    def __del__(self):
        if self._s.value:
            load().rspl_stream_destroy(self._s)
            self._s = C.c_void_p()


class Timer:
    """HIP-event timer recorded on the stream the kernels run on."""

    def __init__(self):
        self._t = C.c_void_p()
        check(load().rspl_timer_create(C.byref(self._t)), "rspl_timer_create")

    def start(self, stream):
        check(load().rspl_timer_record(self._t, 0, stream.handle if isinstance(stream, Stream) else stream), "timer")

    def stop(self, stream):
        check(load().rspl_timer_record(self._t, 1, stream.handle if isinstance(stream, Stream) else stream), "timer")

    def elapsed_ms(self) -> float:
        ms = C.c_float()
        check(load().rspl_timer_elapsed_ms(self._t, C.byref(ms)), "rspl_timer_elapsed_ms")
        return ms.value

    def __del__(self):
        if self._t.value:
            load().rspl_timer_destroy(self._t)
            self._t = C.c_void_p()


def device_count() -> int:
    n = C.c_int(0)
    rc = load().rspl_device_count(C.byref(n))
    return n.value if rc == RSPL_OK else 0


def synchronize():
    check(load().rspl_device_synchronize(), "rspl_device_synchronize")
