"""Map-side local BA on the GPU: the native Map (csrc/map.cpp) with rspl_ba_local inside
Map::LocalMapOptimization (src/map.cc:537-808) against the oracle map (oracle/map_ref.py) with the
oracle's g2o restatement, keyframe by keyframe; then the keyframe trajectory (SaveKeyframeTrajectory)
and its ATE (evo_ape -a restatement) against ground truth and against the oracle's trajectory.
BA tolerances as tests/test_gpu_ba.py (chi2 rtol 1e-8, poses 1e-7); parity unpinned at g2o."""
import numpy as np
import pytest

from conftest import pkg
import oracle
import map_ref
from rspl_slam_amd import synthetic as SY
from rspl_slam_amd import sequence as SQ
from rspl_slam_amd import trajectory as TJ

pytestmark = pytest.mark.gpu


def test_gpu_map_sequence_vs_oracle(tmp_path):
    seq = SY.map_sequence(n_keyframes=16, n_points=2500, n_lines=40, seed=7, outlier_frac=0.05)
    ba = pkg.LocalBA(max_poses=16, max_points=6000, max_lines=200, max_edges=40000)
    mr = map_ref.Map(seq["camera"])
    gpu_reports, orc = [], []

    def check(k, m):
        kf = seq["keyframes"][k]
        map_ref.insert_keyframe(mr, kf)
        if k == 0:
            return
        prob, res, n_out, n_lout = map_ref.local_map_optimization(mr, kf["id"], oracle.ba_local)
        orc.append((res, n_out, n_lout))
        # the GPU flow already ran for keyframe k (sequence.run calls back after it)
        for f in seq["keyframes"][:k + 1]:
            np.testing.assert_allclose(m.GetPose(f["id"]), mr.keyframes[f["id"]].pose, rtol=0, atol=1e-7,
                                       err_msg=f"keyframe {k}: pose {f['id']}")
            assert m.GetOrderedConnections(f["id"]) == mr.keyframes[f["id"]].GetOrderedConnections()

    m, reports = SQ.run(seq, ba, on_keyframe=check)
    assert len(reports) == len(orc) == len(seq["keyframes"]) - 1
    for rep, (res, n_out, n_lout) in zip(reports, orc):
        # a converged optimize() stops when a trial leaves chi2 bit-identical (rho == 0, g2o's stop
        # test); GPU and oracle sum chi2 in different orders, so that last-ulp event can come one
        # iteration apart -- the optimum (chi2, poses) is what must agree
        assert abs(rep["iterations_first"] - res.iters_first) <= 1
        assert abs(rep["iterations_second"] - res.iters_second) <= 1
        np.testing.assert_allclose(rep["chi2_second"], res.chi2_second, rtol=1e-8)
        assert (rep["n_point_outliers"], rep["n_line_outliers"]) == (n_out, n_lout)
    assert sum(r["n_point_outliers"] for r in reports) > 0
    for pid, q in mr.mappoints.items():
        p, t, obs = m.GetMappoint(pid)
        assert t == q.type and obs == q.obs
        np.testing.assert_allclose(p, q.p, rtol=0, atol=1e-6)
    # trajectory: native writer == oracle lines to the printed precision; ATE
    path = tmp_path / "kf.txt"
    m.SaveKeyframeTrajectory(path)
    ts, P, _ = TJ.read_tum(str(path))
    ts_o = np.array([float(l.split()[0]) for l in mr.trajectory_lines()])
    P_o = np.array([[float(v) for v in l.split()[1:4]] for l in mr.trajectory_lines()])
    np.testing.assert_array_equal(ts, ts_o)
    np.testing.assert_allclose(P, P_o, atol=2e-9 + 1e-7)
    gt = seq["gt_Twc"][:, :3, 3]
    tracked = np.array([kf["Twc"][:3, 3] for kf in seq["keyframes"]])
    ate = TJ.ape(seq["timestamps"], gt, ts, P)
    ate_in = TJ.ape(seq["timestamps"], gt, seq["timestamps"], tracked)
    ate_o = TJ.ape(ts_o, P_o, ts, P)
    assert ate_o["rmse"] < 1e-6
    assert ate["rmse"] < 0.5 * ate_in["rmse"], (ate, ate_in)


def test_gpu_map_sequence_analytic_identical_trajectory(tmp_path):
    """Trajectory-level BA parity (round-5 verdict item 1).  With the analytic limit of g2o's central-
    difference line Jacobian on both sides (rspl_ba_set_line_jacobian / oracle.ba_set_line_jacobian) the GPU
    map path and the oracle map path make the same LM decisions on every keyframe, so the keyframe
    trajectories written by SaveKeyframeTrajectory (map.cc:1007-1024) are byte-identical and the poses agree
    to 1e-9 after every keyframe (tools/run_sequence.py --analytic-line-jacobian: identical TUM files over 100
    keyframes, profiles/r06_sequence100_analytic.json).  In g2o's numeric mode the central difference's
    rounding noise (edge_project_line.h:16-31, delta 1e-9) flips an accept / reject decision after ~66
    keyframes and the two paths end mm apart, as two edge orders of the oracle itself do."""
    seq = SY.map_sequence(n_keyframes=48, n_points=4000, n_lines=60, seed=100, outlier_frac=0.03)
    ba = pkg.LocalBA(max_poses=32, max_points=4100, max_lines=70, max_edges=80000)
    ba.set_line_jacobian(True)
    oracle.ba_set_line_jacobian(True)
    try:
        mr = map_ref.Map(seq["camera"])
        iters = []

        def check(k, m):
            kf = seq["keyframes"][k]
            map_ref.insert_keyframe(mr, kf)
            if k == 0:
                return
            _, res, n_out, n_lout = map_ref.local_map_optimization(mr, kf["id"], oracle.ba_local)
            iters.append((res.iters_first, res.iters_second, n_out, n_lout))
            for f in seq["keyframes"][:k + 1]:
                np.testing.assert_allclose(m.GetPose(f["id"]), mr.keyframes[f["id"]].pose, rtol=0, atol=1e-9,
                                           err_msg=f"keyframe {k}: pose {f['id']}")

        m, reports = SQ.run(seq, ba, on_keyframe=check)
    finally:
        ba.set_line_jacobian(False)
        oracle.ba_set_line_jacobian(False)
    assert len(reports) == len(iters) == len(seq["keyframes"]) - 1
    for rep, (i1, i2, n_out, n_lout) in zip(reports, iters):
        assert (rep["iterations_first"], rep["iterations_second"]) == (i1, i2)
        assert (rep["n_point_outliers"], rep["n_line_outliers"]) == (n_out, n_lout)
    assert sum(r["n_line_outliers"] + r["n_point_outliers"] for r in reports) > 0
    assert sum(r["n_lines"] for r in reports) > 0
    path = tmp_path / "kf.txt"
    m.SaveKeyframeTrajectory(path)
    assert path.read_text() == "".join(l + "\n" for l in mr.trajectory_lines())
