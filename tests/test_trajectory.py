"""Dataset I/O, TUM trajectories and evo_ape-style ATE.

Pinned by the reference's own outputs: AirVO_output/oivio/*.txt (copied to tests/golden/tum/) are
trajectories the reference wrote with Map::SaveKeyframeTrajectory (src/map.cc:1007-1024); their
first line is MapBuilder's initial pose (src/map_builder.cc:367-371).  The ATE restates evo's
published algorithm (association, Umeyama SE(3), translation APE) -- evo is not installed, so it
is checked on known answers.
"""
import pathlib

import numpy as np
import pytest

from conftest import pkg
from rspl_slam_amd import trajectory as TJ

GOLD = pathlib.Path(__file__).parent / "golden" / "tum"
FILES = sorted(GOLD.glob("*.txt"))


@pytest.mark.parametrize("path", FILES, ids=[p.name for p in FILES])
def test_tum_roundtrip_reference_files(path):
    ts, p, q = TJ.read_tum(str(path))
    assert len(ts) > 100
    assert TJ.tum_line_strings(ts, p, q) == path.read_text().splitlines()


@pytest.mark.parametrize("path", FILES, ids=[p.name for p in FILES])
def test_tum_writer_reproduces_reference_lines(path):
    """Map::SaveKeyframeTrajectory's quaternion (Eigen Quaterniond(Matrix3d)) of the reference's
    poses re-emits the reference's own lines (last printed digit)."""
    ts, p, q = TJ.read_tum(str(path))
    T = []
    for pi, qi in zip(p, q):
        x, y, z, w = qi / np.linalg.norm(qi)
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                      [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                      [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
        M = np.eye(4)
        M[:3, :3], M[:3, 3] = R, pi
        T.append(M)
    lines = TJ.tum_lines(ts, T)
    ref = path.read_text().splitlines()
    assert lines[0] == ref[0]  # the initial pose, exactly
    a = np.array([[float(v) for v in l.split()] for l in lines])
    b = np.array([[float(v) for v in l.split()] for l in ref])
    np.testing.assert_array_equal(a[:, :4], b[:, :4])
    np.testing.assert_allclose(a[:, 4:], b[:, 4:], atol=2e-9)


def test_initial_pose_line():
    """map_builder.cc:367-371: the first keyframe's T_wc prints as the reference's first line."""
    T = np.array([[1, 0, 0, 0], [0, 0, 1, 0], [0, -1, 0, 1], [0, 0, 0, 1]], np.float64)
    line = TJ.tum_lines([1548880187.382870674], [T])[0]
    assert line == FILES[0].read_text().splitlines()[0]


def _rand_R(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def test_ape_known_answers():
    ts, p, _ = TJ.read_tum(str(FILES[0]))
    rng = np.random.default_rng(0)
    R, t = _rand_R(rng), rng.normal(size=3)
    moved = (R @ p.T).T + t
    r = TJ.ape(ts, p, ts + 0.004, moved, align=True)         # rigid motion + 4 ms stamp offset
    assert r["n"] == len(ts) and r["rmse"] < 1e-9
    assert TJ.ape(ts, p, ts, moved, align=False)["rmse"] > 0.5
    noise = rng.normal(0, 0.01, p.shape)
    r = TJ.ape(ts, p, ts, moved + (R @ noise.T).T, align=True)
    e = np.linalg.norm(noise - noise.mean(0), axis=1)          # alignment absorbs the mean offset
    assert abs(r["rmse"] - np.sqrt(np.mean(e ** 2))) < 2e-4
    # association drops stamps farther than 0.01 s
    off = np.where(np.arange(len(ts)) % 3 == 0, 0.02, 0.003)
    r = TJ.ape(ts, p, ts + off, moved)
    assert r["n"] == int((off <= 0.01).sum()) and r["rmse"] < 1e-9
    with pytest.raises(ValueError):
        TJ.ape(ts[:10], p[:10], ts[:10] + 0.5, p[:10])


def test_umeyama_recovers_transform():
    rng = np.random.default_rng(3)
    x = rng.normal(size=(3, 50))
    R, t = _rand_R(rng), rng.normal(size=3)
    r2, t2, c = TJ.umeyama(x, R @ x + t[:, None], with_scale=False)
    np.testing.assert_allclose(r2, R, atol=1e-12)
    np.testing.assert_allclose(t2, t, atol=1e-12)
    assert c == 1.0


def test_dataset_euroc_layout(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(1)
    names = ["1403636579763555584.png", "1403636579813555456.png", "1403636579863555584.png"]
    imgs = []
    for cam in ("cam0", "cam1"):
        (tmp_path / cam / "data").mkdir(parents=True)
    for n in names[::-1]:  # written out of order: the loader sorts
        a, b = rng.integers(0, 256, (48, 64), dtype=np.uint8), rng.integers(0, 256, (48, 64), dtype=np.uint8)
        Image.fromarray(a, "L").save(tmp_path / "cam0" / "data" / n)
        Image.fromarray(b, "L").save(tmp_path / "cam1" / "data" / n)
        imgs.append((n, a, b))
    ds = TJ.Dataset(str(tmp_path))
    assert ds.GetDatasetLength() == 3
    np.testing.assert_allclose(ds.timestamps, [1403636579.763555584, 1403636579.813555456, 1403636579.863555584],
                               rtol=0, atol=1e-6)
    by = {n: (a, b) for n, a, b in imgs}
    for i, n in enumerate(names):
        d = ds.GetData(i)
        np.testing.assert_array_equal(d["image_left"], by[n][0])
        np.testing.assert_array_equal(d["image_right"], by[n][1])
        assert d["time"] == ds.timestamps[i]
    assert ds.GetData(3) is None
    (tmp_path / "cam1" / "data" / names[1]).unlink()
    assert ds.GetData(1) is None  # FileExists check (dataset.cc:40)


def test_dataset_short_names_use_current_time(tmp_path):
    from PIL import Image
    for cam in ("cam0", "cam1"):
        (tmp_path / cam / "data").mkdir(parents=True)
        Image.fromarray(np.zeros((8, 8), np.uint8), "L").save(tmp_path / cam / "data" / "000001.png")
    ds = TJ.Dataset(str(tmp_path))
    assert ds.timestamps == [] and ds.GetData(0)["time"] > 1.6e9
