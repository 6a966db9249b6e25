"""Load the ``rspl-slam_amd/`` directory as the Python package ``rspl_slam_amd``."""
import importlib.util
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent
PKG_DIR = ROOT / "rspl-slam_amd"


def load():
    if "rspl_slam_amd" in sys.modules:
        return sys.modules["rspl_slam_amd"]
    spec = importlib.util.spec_from_file_location(
        "rspl_slam_amd", PKG_DIR / "__init__.py", submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["rspl_slam_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
