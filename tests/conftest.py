import os
import pathlib
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()
# Load librspl.so (system ROCm HIP runtime) before anything can pull in torch's
# bundled runtime: one HIP runtime per process.
try:
    pkg.capi.load()
except pkg.capi.RsplError:
    pass
GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def weight_blobs():
    from rspl_slam_amd import weights as W
    return W.ensure_blobs(str(ROOT / "weights"))


@pytest.fixture(scope="session")
def sg_c1_blob():
    """SuperGlue weights of the "c1" profile (weights.SG_WEIGHT_GAIN_C1: C1 stereo matches above 0.2)."""
    from rspl_slam_amd import weights as W
    return W.ensure_sg_profile_blob(str(ROOT / "weights"), "c1")


@pytest.fixture(scope="session")
def golden():
    def load(name):
        return np.load(GOLDEN / f"{name}.npz")
    return load
