"""Host staging of the local BA (rspl_ba_debug_stage, csrc/ba_stage.cpp): the caller's four edge
arrays (the reference's constraint vectors, g2o_optimization.cc:81-167) into landmark-CSR order.
Host only -- no device.  Checked against a numpy restatement (a stable sort of the local edges by
landmark, points first) for the serial pass, the host-worker pass (any edge count can be forced onto
the workers with par_edges=1) and the landmark-sharded pass; all three are bit-exact (integers and
copied doubles)."""
import ctypes as C

import numpy as np
import pytest

from rspl_slam_amd import capi
from rspl_slam_amd.ba_types import DenseProblem

KINDS = (("mono", 2), ("stereo", 3), ("mono_line", 4), ("stereo_line", 8))


def _problem(rng, np_, nq, nl, ne, ncam=2, empty_lms=0.0):
    """random dense problem; a fraction of the landmarks gets no edge at all"""
    live_q = np.flatnonzero(rng.random(nq) >= empty_lms) if nq else np.zeros(0, np.int64)
    live_l = np.flatnonzero(rng.random(nl) >= empty_lms) if nl else np.zeros(0, np.int64)
    d = {}
    for (name, od), n in zip(KINDS, ne):
        live = live_q if name in ("mono", "stereo") else live_l
        if not len(live):
            n = 0
        d[name] = dict(pose=rng.integers(0, np_, n), lm=rng.choice(live, n) if n else np.zeros(0),
                       cam=rng.integers(0, ncam, n), obs=rng.standard_normal((n, od)))
    fixed = (rng.random(np_) < 0.2).astype(np.uint8)
    return DenseProblem(cameras=rng.random((ncam, 5)), pose_q=np.tile([0, 0, 0, 1.0], (np_, 1)),
                        pose_p=np.zeros((np_, 3)), pose_fixed=fixed, points=np.zeros((nq, 3)),
                        lines=np.zeros((nl, 6)), **d)


def _expected(p, rank=0, nranks=1):
    nq, nL = p.points.shape[0], p.points.shape[0] + p.lines.shape[0]
    t_all, i_all, g_all = [], [], []
    for t, (name, _) in enumerate(KINDS):
        d = getattr(p, name)
        n = d["pose"].shape[0]
        t_all.append(np.full(n, t))
        i_all.append(np.arange(n))
        g_all.append(d["lm"].astype(np.int64) + (nq if t >= 2 else 0))
    t_all, i_all, g_all = (np.concatenate(a) for a in (t_all, i_all, g_all))
    eg = np.arange(t_all.shape[0])
    keep = (g_all % nranks == rank) if nranks > 1 else np.ones_like(eg, bool)
    order = np.argsort(g_all[keep], kind="stable")
    gmap = eg[keep][order]
    lm_off = np.concatenate([[0], np.cumsum(np.bincount(g_all[keep], minlength=nL))])
    has = np.zeros(p.pose_q.shape[0], bool)
    for name, _ in KINDS:
        has[getattr(p, name)["pose"]] = True
    pidx = np.where(has & (p.pose_fixed == 0), np.cumsum(has & (p.pose_fixed == 0)) - 1, -1)
    return gmap, lm_off, t_all, i_all, g_all, pidx


def _stage(p, par_edges, rank=0, nranks=1):
    lib = capi.load()
    Eg = sum(p.n_edges(k) for k, _ in KINDS)
    nL = p.points.shape[0] + p.lines.shape[0]
    n_local = np.zeros(2, np.int32)
    lm_off = np.full(nL + 1, -7, np.int32)
    etype = np.full(max(Eg, 1), -7, np.int8)
    epose, elm, ecam, gmap, lpose = (np.full(max(Eg, 1), -7, np.int32) for _ in range(5))
    eobs = np.full(8 * max(Eg, 1), np.nan)
    P = p.to_ctypes()
    rc = lib.rspl_ba_debug_stage(C.byref(P), par_edges, rank, nranks, *(a.ctypes.data for a in (
        n_local, lm_off, etype, epose, elm, ecam, gmap, lpose, eobs)))
    return rc, dict(E=int(n_local[0]), Ep=int(n_local[1]), lm_off=lm_off, etype=etype, epose=epose, elm=elm,
                    ecam=ecam, gmap=gmap, lpose=lpose, eobs=eobs)


def _check(p, out, rank=0, nranks=1):
    gmap, lm_off, t_all, i_all, g_all, pidx = _expected(p, rank, nranks)
    E, Ep = out["E"], out["Ep"]
    assert E == gmap.shape[0]
    assert Ep == int(np.sum(t_all[gmap] < 2))
    np.testing.assert_array_equal(out["lm_off"], lm_off)
    np.testing.assert_array_equal(out["gmap"][:E], gmap)
    t, i = t_all[gmap], i_all[gmap]
    np.testing.assert_array_equal(out["etype"][:E], t)
    np.testing.assert_array_equal(out["elm"][:E], g_all[gmap])
    pose = np.array([getattr(p, KINDS[tt][0])["pose"][ii] for tt, ii in zip(t, i)], np.int64).reshape(-1)
    cam = np.array([getattr(p, KINDS[tt][0])["cam"][ii] for tt, ii in zip(t, i)], np.int64).reshape(-1)
    np.testing.assert_array_equal(out["epose"][:E], pose)
    np.testing.assert_array_equal(out["ecam"][:E], cam)
    np.testing.assert_array_equal(out["lpose"][:E], pidx[pose] if E else pose)
    for k in range(E):  # observations copied bit for bit (mono points: third entry 0)
        tt, ii = t[k], i[k]
        ob = getattr(p, KINDS[tt][0])["obs"][ii]
        if tt < 2:
            got = out["eobs"][4 * k:4 * k + 3]
            want = np.array([ob[0], ob[1], ob[2] if tt == 1 else 0.0])
        else:
            got = out["eobs"][4 * Ep + 8 * (k - Ep):4 * Ep + 8 * (k - Ep) + ob.shape[0]]
            want = ob
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("par_edges", [0, 1])
@pytest.mark.parametrize("shape", [
    (10, 400, 30, (300, 500, 40, 60)),     # C3-like, small
    (3, 5, 0, (7, 0, 0, 0)),               # mono points only, fewer landmarks than host workers
    (4, 0, 6, (0, 0, 9, 5)),               # lines only
    (2, 3, 2, (0, 0, 0, 0)),               # no edges
    (1, 1, 1, (1, 1, 1, 1)),
])
def test_stage_matches_numpy(shape, par_edges):
    rng = np.random.default_rng(hash(shape[1:3]) % 2**32)
    p = _problem(rng, shape[0], shape[1], shape[2], shape[3], empty_lms=0.3)
    rc, out = _stage(p, par_edges)
    assert rc == 0, capi.load().rspl_last_error()
    _check(p, out)


def test_stage_workers_equal_serial_at_scale():
    # above the handle's worker threshold (8192 edges): the worker pass against the serial pass
    rng = np.random.default_rng(3)
    p = _problem(rng, 30, 10000, 300, (12000, 18000, 1500, 2500), ncam=3, empty_lms=0.1)
    rc0, a = _stage(p, 0)
    rc1, b = _stage(p, 8192)
    assert rc0 == 0 and rc1 == 0
    assert a["E"] == b["E"] and a["Ep"] == b["Ep"]
    E, Ep = a["E"], a["Ep"]
    np.testing.assert_array_equal(a["lm_off"], b["lm_off"])
    for k in ("etype", "epose", "elm", "ecam", "gmap", "lpose"):
        np.testing.assert_array_equal(a[k][:E], b[k][:E])
    np.testing.assert_array_equal(a["eobs"][4 * Ep:4 * Ep + 8 * (E - Ep)], b["eobs"][4 * Ep:4 * Ep + 8 * (E - Ep)])
    np.testing.assert_array_equal(a["eobs"][:4 * Ep].reshape(-1, 4)[:, :3], b["eobs"][:4 * Ep].reshape(-1, 4)[:, :3])
    _check(p, b)


@pytest.mark.parametrize("nranks", [2, 3])
def test_stage_sharded(nranks):
    rng = np.random.default_rng(nranks)
    p = _problem(rng, 8, 300, 40, (500, 300, 50, 40), empty_lms=0.2)
    total = 0
    for r in range(nranks):
        rc, out = _stage(p, 1, r, nranks)  # sharded calls always stage serially
        assert rc == 0
        _check(p, out, r, nranks)
        total += out["E"]
    assert total == sum(p.n_edges(k) for k, _ in KINDS)


@pytest.mark.parametrize("par_edges", [0, 1])
@pytest.mark.parametrize("bad", ["pose", "lm", "cam"])
def test_stage_rejects_missing_vertex(bad, par_edges):
    rng = np.random.default_rng(5)
    p = _problem(rng, 6, 50, 10, (40, 40, 10, 10))
    d = p.stereo
    d[bad][17] = {"pose": 6, "lm": 50, "cam": 2}[bad]
    p.__dict__.pop("_ct_cache", None)
    rc, _ = _stage(p, par_edges)
    assert rc == -1
    msg = capi.load().rspl_last_error().decode()
    assert "edge 17 of type 1" in msg
