"""N>1 path on CPU: host-group ranks run bench.py's cross-rank timing, census data and replica seeding.

bench.py --gpus N spawns (or torch.distributed.run launches) one process per GPU, each running
its own stereo sequence (replicas, weak scaling).  The host control plane is
rspl-slam_amd/hostgroup.py (TCP on 127.0.0.1, no torch in the rank processes): max-over-ranks wall
time, the rank census, the RCCL id broadcast, rank-ordered host sums.  These tests run that code
(bench.job_time / job_value / replica_seeds / spawn_ranks, api.broadcast_comm_id) in real processes.
"""
import os
import pathlib
import socket
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out):
    sys.path.insert(0, str(ROOT))
    import rspl_loader
    pkg = rspl_loader.load()
    import bench
    g = pkg.hostgroup.HostGroup(rank, world, "127.0.0.1", port, timeout=60)
    try:
        elapsed = 0.5 + rank  # rank 1 is the slow one
        t = bench.job_time(elapsed, g)
        g.barrier()
        x = np.full(5, 0.1 * (rank + 1))
        g.allreduce_sum_(x)
        rows = g.all_gather([rank, rank % 2, 8, "host"])
        out.put((rank, t, bench.job_value(world, 30, t), bench.replica_seeds(rank), x.tolist(), rows))
    finally:
        g.close()


def test_three_rank_host_group_timing_and_replicas():
    """bench.py's N > 1 control plane (hostgroup.HostGroup, no torch): max-over-ranks time seen by every
    rank, whole-job frames/s, disjoint replica seeds, rank-ordered sums bitwise equal on all ranks."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, t, v, seeds, x, rows in res:
        assert t == pytest.approx(2.5)              # max over ranks, seen by every rank
        assert v == pytest.approx(3 * 30 / 2.5)     # whole-job frames/s
        assert rows == [[k, k % 2, 8, "host"] for k in range(3)]
        assert x == res[0][4]                       # identical bits on every rank
    assert res[0][4] == [(0.1 + 0.2) + 0.30000000000000004] * 5
    s = [set(r[3]["images"]) for r in res]
    assert not (s[0] & s[1]) and not (s[1] & s[2])


def test_single_rank_is_identity():
    sys.path.insert(0, str(ROOT))
    import bench
    assert bench.job_time(2.0, None) == 2.0
    assert bench.job_value(1, 10, 2.0) == 5.0


def _id_main(rank, world, port, out):
    sys.path.insert(0, str(ROOT))
    import rspl_loader
    pkg = rspl_loader.load()
    from rspl_slam_amd import api
    g = pkg.hostgroup.HostGroup(rank, world, "127.0.0.1", port, timeout=60)
    try:
        calls = []

        def make_id():  # stands in for rspl_comm_unique_id (RCCL needs a GPU)
            calls.append(rank)
            return bytes(range(128))

        uid = api.broadcast_comm_id(g, make_id)
        out.put((rank, uid, calls))
    finally:
        g.close()


def test_rccl_id_broadcast_two_ranks():
    """The sharded BA's RCCL bootstrap (api.broadcast_comm_id): only rank 0 makes the id, every
    rank of the gloo group receives the same 128 bytes."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_id_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, u0, c0), (r1, u1, c1) = res
    assert u0 == u1 == bytes(range(128))
    assert c0 == [0] and c1 == []


RANK_SCRIPT = """
import os, sys, time, pathlib
out = pathlib.Path(sys.argv[1])
r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
(out / f"rank{r}").write_text(f"{r} {w} {os.environ['LOCAL_RANK']} {os.environ['MASTER_ADDR']}")
if len(sys.argv) > 2 and r == int(sys.argv[2]):
    sys.exit(3)                   # this rank fails
if len(sys.argv) > 2:
    time.sleep(600)               # the others would wait for it forever
"""


def test_spawn_ranks(tmp_path):
    """bench.py --gpus N without a launcher: N rank processes with RANK / WORLD_SIZE / LOCAL_RANK and a
    127.0.0.1 rendezvous; a failing rank ends the job with its exit code (the others are killed)."""
    sys.path.insert(0, str(ROOT))
    import time
    import bench
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    assert bench.spawn_ranks(3, [str(tmp_path)], script=script) == 0
    rows = sorted((tmp_path / f"rank{r}").read_text() for r in range(3))
    assert rows == [f"{r} 3 {r} 127.0.0.1" for r in range(3)]
    t = time.time()
    assert bench.spawn_ranks(2, [str(tmp_path), "1"], script=script) == 3
    assert time.time() - t < 60
