"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

Corrections per MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KB; on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced read, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane stores.  Usage:
    python tools/pmc_traffic.py FETCH.csv WRITE.csv [kernel-substring ...] > profiles/...json
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    pats = sys.argv[3:] or [""]
    out = {}
    for name in sorted(set(fetch) & set(write)):
        if not any(p in name for p in pats):
            continue
        f = sum(fetch[name]) / len(fetch[name]) * 1024 * 2  # KB -> B, x2 gfx950 read correction
        w = sum(write[name]) / len(write[name]) * 1024
        out[name] = {"launches": len(fetch[name]), "read_bytes": f, "write_bytes": w, "traffic_bytes": f + w}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
