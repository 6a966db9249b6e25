"""N>1 path on CPU: world_size-2 gloo ranks run bench.py's cross-rank timing and replica seeding.

bench.py --gpus N is launched by torch.distributed.run, one process per GPU, each running
its own stereo sequence (replicas, weak scaling).  The only collective is the max-over-ranks
wall time; this test exercises exactly that code (bench.job_time / job_value / replica_seeds)
with two real gloo processes on 127.0.0.1.
"""
import os
import pathlib
import socket
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        elapsed = 0.5 + rank  # rank 1 is the slow one
        t = bench.job_time(elapsed, dist)
        dist.barrier()
        out.put((rank, t, bench.job_value(world, 30, t), bench.replica_seeds(rank)))
    finally:
        dist.destroy_process_group()


def test_two_rank_timing_and_replicas():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, t0, v0, s0), (r1, t1, v1, s1) = res
    assert t0 == t1 == pytest.approx(1.5)           # max over ranks, seen by every rank
    assert v0 == v1 == pytest.approx(2 * 30 / 1.5)   # whole-job frames/s
    # replicas: disjoint synthetic sequences per rank
    assert not set(s0["images"]) & set(s1["images"])
    assert not set(s0["ba"]) & set(s1["ba"])


def test_single_rank_is_identity():
    sys.path.insert(0, str(ROOT))
    import bench
    assert bench.job_time(2.0, None) == 2.0
    assert bench.job_value(1, 10, 2.0) == 5.0


def _id_main(rank, world, port, out):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import rspl_loader
    pkg = rspl_loader.load()
    from rspl_slam_amd import api
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = []

        def make_id():  # stands in for rspl_comm_unique_id (RCCL needs a GPU)
            calls.append(rank)
            return bytes(range(128))

        uid = api.broadcast_comm_id(dist, make_id)
        out.put((rank, uid, calls))
    finally:
        dist.destroy_process_group()


def test_rccl_id_broadcast_two_ranks():
    """The sharded BA's RCCL bootstrap (api.broadcast_comm_id): only rank 0 makes the id, every
    rank of the gloo group receives the same 128 bytes."""
    import torch.multiprocessing as mp
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
