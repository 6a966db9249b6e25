"""Host-side mirror of the reference's C++ classes for the hot path, over the C ABI.

  SuperPoint     include/super_point.h:20-66      (build / infer)
  SuperGlue      include/super_glue.h:20-71       (build / infer)
  PointMatching  include/point_matching.h:7-18    (MatchingPoints / NormalizeKeypoints)
  LocalmapOptimization  include/g2o_optimization/g2o_optimization.h:15-19

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
        """SuperPoint::infer (src/super_point.cpp:174-205): u8 [H, W] -> (ok, features [259, N])."""
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

    def debug_maps(self, b: int, height: int, width: int):
        s = np.empty((height, width), np.float32)
        d = np.empty((256, height // 8, width // 8), np.float32)
        capi.check(self._lib.rspl_sp_debug_maps(self._h, b, s.ctypes.data, d.ctypes.data), "rspl_sp_debug_maps")
        return s, d

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            self._lib.rspl_sp_destroy(self._h)
            self._h = C.c_void_p()
