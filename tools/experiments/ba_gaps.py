"""Host-induced gaps of the local BA's HW queue in a rocprofv3 kernel-trace CSV: per call, the idle time
at the call boundary (finish -> next call's first kernel), at the optimize(10) -> optimize(5) hand-over
and between an optimize's first kernels (setup -> first Schur chunk)."""
import collections
import csv
import glob
import sys

import numpy as np


def main():
    path = sys.argv[1]
    if not path.endswith(".csv"):
        path = sorted(glob.glob(path + "/**/*kernel_trace.csv", recursive=True))[0]
    rows = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        rows[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                    r["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0]))
    q = max(rows, key=lambda k: sum(1 for x in rows[k] if x[2] == "pair_chunk_kernel"))
    ba = sorted(rows[q])
    bound, hand, first, busy, span = [], [], [], 0.0, 0.0
    for i, (s, e, n) in enumerate(ba):
        if n != "setup_kernel" or i == 0:
            continue
        g = (s - ba[i - 1][1]) / 1e3
        (bound if ba[i - 1][2] == "finish_kernel" else hand).append(g)
        j = i + 1
        while j < len(ba) and ba[j][2] != "pair_chunk_kernel":
            j += 1
        if j < len(ba):
            first.append((ba[j][0] - e) / 1e3)
    calls = [i for i, r in enumerate(ba) if r[2] == "finish_kernel"]
    for a, b in zip(calls[len(calls) // 4:], calls[len(calls) // 4 + 1:]):
        busy += sum(ba[k][1] - ba[k][0] for k in range(a + 1, b + 1)) / 1e3
        span += (ba[b][1] - ba[a][1]) / 1e3
    n = len(calls) - len(calls) // 4 - 1
    p = lambda v: np.percentile(v, [10, 50, 90]).round(1).tolist() if v else None
    print(f"calls {len(calls)}: per call {span / max(n, 1):.1f} us, BA kernels busy {busy / max(n, 1):.1f} us; "
          f"call boundary gap p10/50/90 {p(bound)}; opt10->opt5 {p(hand)}; setup end -> first chunk {p(first)}")


if __name__ == "__main__":
    main()
