"""rspl_slam_amd -- MI355X-native SuperPoint -> SuperGlue -> local-BA hot path.

Loaded by path as the module ``rspl_slam_amd`` (see rspl_loader.py; the
directory name carries a dash).  The compute path is librspl.so (HIP, gfx950);
this package only mirrors the reference's C++ interface over its C ABI.
"""
import importlib

from . import capi, weights, synthetic, ba_types, hostgroup, mapping, trajectory, sequence, lines  # noqa: F401

_API = ("SuperPoint", "SuperPointConfig", "SuperGlue", "SuperGlueConfig", "PointMatching",
        "LocalmapOptimization", "LocalBA", "FrameOptimization", "FrameBA",
        "ShardGroup", "Comm", "comm_unique_id", "broadcast_comm_id", "PnP", "SolvePnPWithCV")


def __getattr__(name):
    # the API module is imported lazily so CPU-only tooling (weights, synthetic) never loads librspl.so
    if name in _API:
        return getattr(importlib.import_module(__name__ + ".api"), name)
    raise AttributeError(name)
