"""Keyframe sequence driver for the map-side local BA: what MapBuilder does with each new keyframe
once tracking has produced it -- Map::InsertKeyframe's bookkeeping (src/map.cc:24-103) followed
by Map::LocalMapOptimization (:105-107) on the GPU -- and the trajectory it leaves
(Map::SaveKeyframeTrajectory, :1007-1024).  Input: synthetic.map_sequence (tracking output with
ground truth).  Tracking, keyframe selection and landmark triangulation are not on this path.
"""
from __future__ import annotations

import time

import numpy as np

from .ba_types import OptimizationConfig
from .mapping import Map


def insert_keyframe(m: Map, kf: dict):
    """Map::InsertKeyframe bookkeeping: the frame, its new landmarks, every observation."""
    m.InsertKeyframe(kf["id"], kf["timestamp"], kf["Twc"], kf["keypoints"], kf["lines_left"], kf["lines_right"],
                     kf["lines_right_valid"], kf["points_on_lines"], kf["parent_id"])
    if kf["new_points"]:
        m.InsertMappoints([i for i, _ in kf["new_points"]], np.array([p for _, p in kf["new_points"]]))
    for i, L in kf["new_lines"]:
        m.InsertMapline(i, L)
    if kf["point_obs"]:
        ob = np.array(kf["point_obs"], np.int32)
        m.AddPointObservations(kf["id"], ob[:, 0], ob[:, 1])
    for i, j in kf["line_obs"]:
        m.AddLineObservation(i, kf["id"], j)


def run(seq: dict, ba, cfg: OptimizationConfig = OptimizationConfig(), iterations=(10, 5), on_keyframe=None):
    """Every keyframe of `seq` into a new Map, with LocalMapOptimization (GPU BA handle `ba`) from the
    second keyframe on.  Returns (map, per-keyframe reports)."""
    m = Map(seq["camera"], cfg, iterations)
    reports = []
    for k, kf in enumerate(seq["keyframes"]):
        t = time.perf_counter()
        insert_keyframe(m, kf)
        t_ins = time.perf_counter() - t
        if k >= 1:  # map.cc:29 (the first keyframe only initialises) and :105-107
            r = m.LocalMapOptimization(kf["id"], ba)
            r["insert_us"] = 1e6 * t_ins  # the keyframe's bookkeeping through the Python API
            reports.append(r)
        if on_keyframe:
            on_keyframe(k, m)
    return m, reports


def keyframe_trajectory(m: Map, seq: dict) -> np.ndarray:
    """[n][4][4] current keyframe poses T_wc in insertion order."""
    return np.array([m.GetPose(kf["id"]) for kf in seq["keyframes"]])
