"""Host launch lag of the local BA's kernels in a rocprofv3 --kernel-trace --hip-trace run (CSV): for every BA
kernel, the time from the end of its host launch call to the kernel's start, and how much of the idle gap
before the kernel (previous BA kernel's end -> its start) the host caused (the launch call ended after the
previous kernel had finished).  Split by transition kind as tools/experiments/ba_chain.py."""
import collections
import csv
import glob
import sys

import numpy as np


def short(n):
    return n.split("(")[0].split("::")[-1].split("<")[0]


def main():
    d = sys.argv[1]
    kt = sorted(glob.glob(d + "/**/*kernel_trace.csv", recursive=True))[0]
    ht = sorted(glob.glob(d + "/**/*hip_api_trace.csv", recursive=True))[0]
    launch = {}
    for r in csv.DictReader(open(ht)):
        if "Launch" in r["Function"]:
            launch[r["Correlation_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Thread_Id"])
    rows = collections.defaultdict(list)
    for r in csv.DictReader(open(kt)):
        rows[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                                    r["Correlation_Id"]))
    q = max(rows, key=lambda k: sum(1 for x in rows[k] if x[2] == "pair_chunk_kernel"))
    ba = sorted(rows[q])
    n0 = len(ba) // 4
    gap_by = collections.defaultdict(list)
    host_by = collections.defaultdict(list)
    lag_by = collections.defaultdict(list)
    nset = 0
    for i in range(1, len(ba)):
        s, e, n, cid = ba[i]
        prev = ba[i - 1]
        if n == "setup_kernel":
            nset += 1
        if i < n0:
            continue
        if n == "setup_kernel":
            key = "setup"
        elif n == "pair_chunk_kernel" and prev[2] in ("setup_kernel", "pair_fill_kernel"):
            key = "first chunks"
        elif n == "pair_chunk_kernel":
            key = "chunks (trial)"
        elif n.startswith("update_errors"):
            key = "update"
        else:
            key = n
        gap = (s - prev[1]) / 1e3
        L = launch.get(cid)
        if L is None:
            continue
        host_late = max(0.0, min(gap, (L[1] - prev[1]) / 1e3))  # the part of the gap before the launch returned
        gap_by[key].append(gap)
        host_by[key].append(host_late)
        lag_by[key].append((s - L[1]) / 1e3)
    # host side: launch-call durations per thread, and on the BA thread the host time from one launch call's
    # end to the next one's start (what the tracking thread did between two launches), by the kernel launched
    by_thread = collections.defaultdict(list)
    for cid, (a, b_, t) in launch.items():
        by_thread[t].append((a, b_, cid))
    kname = {x[3]: x[2] for x in ba}
    ba_thread = collections.Counter(launch[x[3]][2] for x in ba if x[3] in launch).most_common(1)[0][0]
    for t, L in by_thread.items():
        d = np.array([(b_ - a) / 1e3 for a, b_, _ in L])
        print(f"thread {t}{' (BA)' if t == ba_thread else ''}: {len(L)} launch calls, duration p50 {np.median(d):.2f} "
              f"p90 {np.percentile(d, 90):.2f} max {d.max():.1f} us")
    L = sorted(by_thread[ba_thread])
    between = collections.defaultdict(list)
    for (a0, b0, c0), (a1, b1, c1) in zip(L, L[1:]):
        between[f"{kname.get(c0, '?')} -> {kname.get(c1, '?')}"].append((a1 - b0) / 1e3)
    print("BA thread, host time between consecutive launch calls (us, p50 / mean / n):")
    for k, v in sorted(between.items(), key=lambda x: -np.mean(x[1]) * len(x[1]))[:12]:
        print(f"  {k:45s} {np.median(v):8.2f} {np.mean(v):8.2f} {len(v):6d}")
    print(f"{'kernel':16s} {'n':>6s} {'gap mean':>9s} {'host-late mean':>15s} {'launch->start p50':>18s}")
    for k in gap_by:
        print(f"{k:16s} {len(gap_by[k]):6d} {np.mean(gap_by[k]):9.2f} {np.mean(host_by[k]):15.2f} "
              f"{np.median(lag_by[k]):18.2f}")


if __name__ == "__main__":
    main()
