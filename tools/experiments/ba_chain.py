"""Where a local-BA call's wall time goes in a rocprofv3 kernel trace of the bench (--kernel-trace CSV): per
call, the BA queue's kernel busy time by kind and the idle gaps by transition (upload -> setup, setup ->
first chunks, chunks -> update inside a trial, update -> next chunks between trials, the optimize(10) ->
optimize(5) hand-over, last trial -> finish).  Medians over the calls after the first quarter (warm)."""
import collections
import csv
import glob
import sys

import numpy as np


def short(n):
    return n.split("(")[0].split("::")[-1].split("<")[0]


def main():
    path = sys.argv[1]
    if not path.endswith(".csv"):
        path = sorted(glob.glob(path + "/**/*kernel_trace.csv", recursive=True))[0]
    rows = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        rows[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    q = max(rows, key=lambda k: sum(1 for x in rows[k] if x[2] == "pair_chunk_kernel"))
    ba = sorted(rows[q])
    # split into calls at each finish_kernel
    calls, cur = [], []
    for k in ba:
        cur.append(k)
        if k[2] == "finish_kernel":
            calls.append(cur)
            cur = []
    calls = calls[len(calls) // 4:]
    busy = collections.defaultdict(list)
    gaps = collections.defaultdict(list)
    spans, trials = [], []
    for c in calls:
        spans.append((c[-1][1] - c[0][0]) / 1e3)
        b = collections.Counter()
        g = collections.Counter()
        nset = 0
        for i, (s, e, n) in enumerate(c):
            b[n] += (e - s) / 1e3
            if i == 0:
                continue
            prev = c[i - 1][2]
            gap = (s - c[i - 1][1]) / 1e3
            if n == "setup_kernel":
                nset += 1
                key = "-> setup (opt1)" if nset == 1 else "opt10 -> opt5 (-> setup)"
            elif n == "pair_chunk_kernel" and prev in ("setup_kernel", "pair_fill_kernel"):
                key = "setup -> first chunks"
            elif n == "pair_chunk_kernel":
                key = "update -> chunks (between trials)"
            elif n.startswith("update_errors"):
                key = "chunks -> update (in trial)"
            elif n == "finish_kernel":
                key = "-> finish"
            else:
                key = f"{prev} -> {n}"
            g[key] += gap
        trials.append(sum(1 for x in c if x[2] == "pair_chunk_kernel"))
        for k, v in b.items():
            busy[k].append(v)
        for k, v in g.items():
            gaps[k].append(v)
    med = lambda v: float(np.median(v))
    print(f"{len(calls)} warm calls; span median {med(spans):.1f} us, trials per call {med(trials):.0f}")
    print("busy (us per call):", {k: round(med(v), 1) for k, v in sorted(busy.items(), key=lambda x: -med(x[1]))})
    print("busy total", round(med([sum(x) for x in zip(*busy.values())]) if busy else 0, 1))
    print("gaps (us per call):", {k: round(med(v), 1) for k, v in sorted(gaps.items(), key=lambda x: -med(x[1]))})
    print("gaps total", round(sum(med(v) for v in gaps.values()), 1))


if __name__ == "__main__":
    main()
