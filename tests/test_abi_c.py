"""The C ABI from C: tests/c/abi_consumer.c includes include/rspl.h and links librspl.so with gcc.

CPU: every struct's sizeof / offsetof as the C compiler lays it out equals the ctypes mirrors the
Python side uses (rspl-slam_amd/capi.py, ba_types.py) -- a layout slip can no longer hit both sides
alike unnoticed.  GPU: the C program runs rspl_sp_infer, rspl_sg_infer, rspl_pm_match and
rspl_ba_local on small fixtures and its outputs match the reference fixtures / the oracle."""
import ctypes as C
import json
import pathlib
import subprocess

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
EXE = ROOT / "tests" / "c" / "build" / "abi_consumer"


def _exe():
    if not EXE.exists():
        subprocess.run(["make", "-C", str(ROOT / "tests" / "c")], check=True, capture_output=True)
    return EXE


def _mirrors():
    import rspl_loader
    pkg = rspl_loader.load()
    from rspl_slam_amd import ba_types as BT
    capi = pkg.capi
    return {"rspl_sp_config": capi.SpConfig, "rspl_sg_config": capi.SgConfig, "rspl_dmatch": capi.DMatch,
            "rspl_ba_config": capi.BaConfig, "rspl_ba_problem": BT.RsplBaProblem, "rspl_ba_result": BT.RsplBaResult,
            "rspl_frame_config": capi.FrameConfig, "rspl_frame_problem": BT.RsplFrameProblem,
            "rspl_frame_result": BT.RsplFrameResult, "rspl_pnp_config": capi.PnpConfig,
            "rspl_pnp_problem": capi.PnpProblem, "rspl_pnp_result": capi.PnpResult,
            "rspl_map_config": pkg.mapping.MapConfig, "rspl_map_keyframe": pkg.mapping.MapKeyframe,
            "rspl_map_report": pkg.mapping.MapReport, "rspl_lines_config": pkg.lines.LinesConfig}


def test_struct_layout_matches_ctypes():
    got = json.loads(subprocess.run([str(_exe()), "layout"], check=True, capture_output=True, text=True).stdout)
    mirrors = _mirrors()
    assert set(got) == set(mirrors)
    for name, T in mirrors.items():
        assert got[name]["size"] == C.sizeof(T), name
        cfields = [f[0] for f in T._fields_]
        assert list(got[name]["fields"]) == cfields, name          # same fields, same order
        for f, off in got[name]["fields"].items():
            assert getattr(T, f).offset == off, f"{name}.{f}"


@pytest.mark.gpu
def test_c_consumer_runs_the_hot_path(tmp_path, golden, weight_blobs):
    import oracle
    import post
    from helpers import compare_features
    from rspl_slam_amd import synthetic as SY
    # SuperPoint fixture (reference module outputs, convert2onnx/superpoint.py)
    g = golden("sp_small")
    img = np.ascontiguousarray(g["image"], np.uint8)
    with open(tmp_path / "sp_in.bin", "wb") as f:
        f.write(np.array([img.shape[0], img.shape[1], 32, 4], np.int32).tobytes())
        f.write(np.array([0.004], np.float64).tobytes())
        f.write(img.tobytes())
    # SuperGlue / PointMatching fixture (raw features; the C side normalises for rspl_sg_infer)
    s = golden("sg_400")
    F0, F1 = s["F0"].astype(np.float64), s["F1"].astype(np.float64)
    with open(tmp_path / "sg_in.bin", "wb") as f:
        f.write(np.array([F0.shape[1], F1.shape[1], 752, 480], np.int32).tobytes())
        f.write(np.ascontiguousarray(F0.T).tobytes())
        f.write(np.ascontiguousarray(F1.T).tobytes())
    # local BA: small synthetic problem with lines, checked against the fp64 restatement
    prob, _ = SY.ba_problem(n_poses=6, n_points=300, n_lines=12, seed=8, pixel_sigma=0.8, outlier_frac=0.05)
    sets = (("mono", 2), ("stereo", 3), ("mono_line", 4), ("stereo_line", 8))
    with open(tmp_path / "ba_in.bin", "wb") as f:
        f.write(np.array([len(prob.cameras), len(prob.pose_q), len(prob.points), len(prob.lines)] +
                         [prob.n_edges(n) for n, _ in sets] + [prob.iterations_first, prob.iterations_second],
                         np.int32).tobytes())
        c = prob.cfg
        f.write(np.array([c.mono_point, c.stereo_point, c.mono_line, c.stereo_line], np.float64).tobytes())
        for a in (prob.cameras, prob.pose_q, prob.pose_p, prob.pose_fixed, prob.points, prob.lines):
            f.write(np.ascontiguousarray(a).tobytes())
        for n, _ in sets:
            d = getattr(prob, n)
            for k in ("pose", "lm", "cam", "obs"):
                f.write(np.ascontiguousarray(d[k]).tobytes())
    sp_w, sg_w = weight_blobs
    r = subprocess.run([str(_exe()), "run", str(tmp_path), sp_w, sg_w], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    # SuperPoint
    raw = (tmp_path / "sp_out.bin").read_bytes()
    n = int(np.frombuffer(raw[:4], np.int32)[0])
    Fsp = np.frombuffer(raw[4:], np.float64).reshape(n, 259).T
    compare_features(Fsp, g["features"])
    # SuperGlue + PointMatching
    raw = (tmp_path / "sg_out.bin").read_bytes()
    n0, n1 = F0.shape[1], F1.shape[1]
    o = 0
    i0 = np.frombuffer(raw, np.int32, n0, o); o += 4 * n0
    i1 = np.frombuffer(raw, np.int32, n1, o); o += 4 * n1
    m0 = np.frombuffer(raw, np.float64, n0, o); o += 8 * n0
    o += 8 * n1
    nm = int(np.frombuffer(raw, np.int32, 1, o)[0]); o += 4
    mt = np.frombuffer(raw, np.dtype([("q", "<i4"), ("t", "<i4"), ("d", "<f4")]), nm, o)
    np.testing.assert_array_equal(i0, s["idx0"])
    np.testing.assert_array_equal(i1, s["idx1"])
    np.testing.assert_allclose(m0, s["ms0"], rtol=1e-4, atol=1e-6)
    np.testing.assert_array_equal(np.stack([mt["q"], mt["t"]], 1), s["matches"])
    np.testing.assert_allclose(mt["d"], s["distances"], atol=1e-5)
    # local BA
    raw = (tmp_path / "ba_out.bin").read_bytes()
    chi2 = np.frombuffer(raw, np.float64, 2, 0)
    its = np.frombuffer(raw, np.int32, 2, 16)
    o = 24
    npo, nq, nl = len(prob.pose_q), len(prob.points), len(prob.lines)
    q = np.frombuffer(raw, np.float64, 4 * npo, o).reshape(npo, 4); o += 32 * npo
    p = np.frombuffer(raw, np.float64, 3 * npo, o).reshape(npo, 3); o += 24 * npo
    X = np.frombuffer(raw, np.float64, 3 * nq, o).reshape(nq, 3); o += 24 * nq
    o += 48 * nl
    ref = oracle.ba_local(prob)
    assert (int(its[0]), int(its[1])) == (ref.iters_first, ref.iters_second)
    np.testing.assert_allclose(chi2, [ref.chi2_first, ref.chi2_second], rtol=1e-8)
    assert np.abs(p - ref.pose_p).max() < 1e-7 and np.abs(X - ref.points).max() < 1e-6
    for n, _ in sets:
        k = prob.n_edges(n)
        np.testing.assert_array_equal(np.frombuffer(raw, np.uint8, k, o), ref.inlier[n], err_msg=n)
        o += k
    assert q.shape == (npo, 4)
