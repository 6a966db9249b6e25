"""Landmark-sharded local BA timing.

  python tools/bench_ba_shard.py                       # one GPU: unsharded vs in-process groups of G ranks
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/bench_ba_shard.py --rccl
                                                       # N GPUs, one rank each, RCCL all-reduce over xGMI
Workloads: C5 (30 poses / 1 fixed, 10k points, 5 % outliers) and C3 (10 poses, 4k points, 100 lines).
Prints one JSON line (rank 0)."""
import argparse
import json
import os
import pathlib
import sys
import threading
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import rspl_loader  # noqa: E402

pkg = rspl_loader.load()
pkg.capi.load()

WORKLOADS = {"C5": dict(n_poses=30, n_points=10000, n_lines=0, seed=5),
             "C3": dict(n_poses=10, n_points=4000, n_lines=100, seed=7)}
CAPS = (40, 12000, 400, 80000)


def timed(fn, iters):
    fn()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    return (time.perf_counter() - t) / iters * 1e3


def group_run(prob, G, iters):
    group = pkg.ShardGroup(G)
    bas = [pkg.LocalBA(*CAPS) for _ in range(G)]
    for r, b in enumerate(bas):
        b.set_group(group, r)

    def once():
        th = [threading.Thread(target=bas[r].run, args=(prob,)) for r in range(G)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    return timed(once, iters)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rccl", action="store_true")
    ap.add_argument("--groups", default="1,2,4")
    a = ap.parse_args()
    out = {}
    probs = {k: pkg.synthetic.ba_problem(pixel_sigma=0.8, outlier_frac=0.05, **v)[0] for k, v in WORKLOADS.items()}
    if a.rccl:
        import torch.distributed as dist
        rank, world, local = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ["LOCAL_RANK"])
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pkg.capi.check(pkg.capi.load().rspl_set_device(local), "rspl_set_device")
        comm = pkg.Comm(pkg.broadcast_comm_id(dist), rank, world, local)
        ba = pkg.LocalBA(*CAPS, device=local)
        ba.set_comm(comm)
        for k, p in probs.items():
            dist.barrier()
            ms = timed(lambda: ba.run(p), a.iters)
            import torch
            t = torch.tensor([ms], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            out[f"{k}_rccl_x{world}_ms"] = round(float(t[0]), 3)
        if rank == 0:
            print(json.dumps(out), flush=True)
        dist.destroy_process_group()
        return
    for k, p in probs.items():
        plain = pkg.LocalBA(*CAPS)
        out[f"{k}_unsharded_ms"] = round(timed(lambda: plain.run(p), a.iters), 3)
        for G in [int(g) for g in a.groups.split(",")]:
            out[f"{k}_group_x{G}_ms"] = round(group_run(p, G, a.iters), 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
