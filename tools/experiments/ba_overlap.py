"""Which front-end kernels slow the local BA down in the pipeline?  Reads a rocprofv3 kernel-trace CSV
(`--kernel-trace --output-format csv`) of bench.py and, for every BA trial kernel (pair_chunk /
update_errors), finds the front-end kernels that overlap it in time.  Prints, per BA kernel, the mean
duration alone vs. overlapped by each front-end kernel class (the class's share of the BA kernel's span),
and the BA's per-call timeline: kernel busy time vs. the gaps between its launches."""
import collections
import csv
import glob
import sys

import numpy as np


def kclass(name):
    n = name.split("(")[0]
    for key, cls in (("rspl::ba::", None), ("conv3x3", "sp:conv"), ("layer_kernel", "sg:gnn"), ("sinkhorn", "sg:sinkhorn"),
                     ("nms", "sp:nms"), ("topk", "sp:topk"), ("sample", "sp:sample"), ("det_head", "sp:head"),
                     ("canny", "lines:canny"), ("assign", "lines:assoc"), ("match_kernel", "lines:assoc"),
                     ("gemm", "sg:gemm"), ("kenc", "sg:kenc"), ("prep", "sg:prep"), ("argmax", "sg:decode"),
                     ("finalize", "sg:decode"), ("bins", "sg:sinkhorn")):
        if key in n:
            return cls if cls else "ba:" + n.split("rspl::ba::")[1].split("<")[0].split("(")[0]
    return "other:" + n[:40]


def main():
    path = sys.argv[1]
    if not path.endswith(".csv"):
        path = sorted(glob.glob(path + "/**/*kernel_trace.csv", recursive=True))[0]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kclass(r["Kernel_Name"])))
    rows.sort()
    # the last half of the run (timed region of a short bench; warmup / fp32 runs excluded by the caller)
    t_lo = rows[len(rows) // 3][0]
    ba = [r for r in rows if r[2].startswith("ba:") and r[0] >= t_lo]
    fe = [r for r in rows if not r[2].startswith("ba:")]
    fe_s = np.array([r[0] for r in fe])
    stats = collections.defaultdict(lambda: collections.defaultdict(list))
    for s, e, c in ba:
        dur = (e - s) / 1e3
        # front-end kernels overlapping [s, e): started before e, ended after s
        i1 = np.searchsorted(fe_s, e)
        share = collections.Counter()
        for fs, fe_, fc in fe[max(0, i1 - 400):i1]:
            if fe_ > s:
                share[fc] += (min(e, fe_) - max(s, fs)) / max(e - s, 1)
        stats[c]["all"].append(dur)
        if not share:
            stats[c]["alone"].append(dur)
        for fc, sh in share.items():
            if sh > 0.5:
                stats[c][fc].append(dur)
    for c in sorted(stats):
        d = stats[c]
        print(f"{c}: n {len(d['all'])} mean {np.mean(d['all']):.2f} us median {np.median(d['all']):.2f}"
              f" alone {np.mean(d['alone']) if d['alone'] else float('nan'):.2f} us (n {len(d['alone'])})")
        for fc in sorted(d, key=lambda k: -len(d[k])):
            if fc in ("all", "alone"):
                continue
            print(f"    overlapped >50% by {fc:16s} n {len(d[fc]):5d} mean {np.mean(d[fc]):7.2f} us")
    # BA busy vs gap: between consecutive BA kernels
    gaps = [(ba[i + 1][0] - ba[i][1]) / 1e3 for i in range(len(ba) - 1)]
    g = np.array(gaps)
    print(f"BA inter-kernel gaps: median {np.median(g):.2f} us, <10us mean {g[g < 10].mean():.2f} (n {(g < 10).sum()}),"
          f" 10-200us n {((g >= 10) & (g < 200)).sum()} sum {g[(g >= 10) & (g < 200)].sum() / 1e3:.2f} ms,"
          f" span {(ba[-1][1] - ba[0][0]) / 1e6:.2f} ms, BA kernel busy {sum(e - s for s, e, _ in ba) / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
