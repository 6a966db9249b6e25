"""Rank body of tests/test_gpu_ba_shard.py::test_two_process_shard_host_allreduce (a module of its own, so a
spawned process can import it without the test module's package imports)."""
import pathlib
import sys


def rank_main(rank, world, port, q, prob_kw):
    """One process of the 2-process sharded BA: its own HIP runtime and rspl_ba handle on GPU 0,
    the per-trial all-reduces host-staged over the TCP host group (no torch in the
    process: one HIP runtime)."""
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root))
    try:
        import rspl_loader
        pkg = rspl_loader.load()
        pkg.capi.load()
        group = pkg.hostgroup.HostGroup(rank, world, "127.0.0.1", port, timeout=60)
        prob, _ = pkg.synthetic.ba_problem(**prob_kw)
        ba = pkg.LocalBA(16, 2000, 64, 20000)
        ba.set_shard(rank, world, group.allreduce_sum_)
        r = ba.run(prob)
        q.put((rank, r.iters_first, r.iters_second, r.chi2_first, r.chi2_second, r.pose_q, r.pose_p, r.points,
               r.lines, {k: v.copy() for k, v in r.inlier.items()}))
        group.close()
    except Exception as e:  # reported to the parent
        q.put((rank, "error", repr(e)))
