"""CPU-side checks of the boundary: librspl.so loads and exports every symbol
include/rspl.h declares (no compute calls -- there is no GPU here)."""
import pathlib
import re

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _declared():
    hdr = (ROOT / "include" / "rspl.h").read_text()
    return sorted(set(re.findall(r"\b(rspl_[a-z0-9_]+)\s*\(", hdr)))


def test_header_declares_api():
    names = _declared()
    for n in ("rspl_sp_create", "rspl_sp_infer", "rspl_sg_infer", "rspl_pm_match", "rspl_ba_local", "rspl_last_error"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from rspl_slam_amd import capi
    lib = capi.load()
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, f"librspl.so lacks {missing}"
    assert b"gfx950" in lib.rspl_version()


def test_no_cpu_fallback_when_library_missing(tmp_path):
    from rspl_slam_amd import capi
    with pytest.raises(capi.RsplError):
        capi._lib_backup = capi._lib
        capi._lib = None
        try:
            capi.load(tmp_path / "nope.so")
        finally:
            capi._lib = capi._lib_backup


def test_create_rejects_bad_config(weight_blobs):
    import rspl_loader
    pkg = rspl_loader.load()
    sp = pkg.SuperPoint(pkg.SuperPointConfig(weights=weight_blobs[0], max_height=100, max_width=752))
    assert not sp.build()           # 100 is not a multiple of 8: rejected before touching a device
    assert "multiples of 8" in sp.error
