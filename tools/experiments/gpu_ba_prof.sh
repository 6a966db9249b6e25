#!/bin/bash
# Standalone C3 BA: time per call and the median in-kernel trial trace (RSPL_BA_PROF)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/bench_ba.py --iters 30 || exit 1
RSPL_BA_PROF=1 timeout -k 10 120 python -u tools/bench_ba.py --iters 20 > /dev/null 2> gpurun_out/bprof.err || exit 1
python3 - <<'PY'
import re, numpy as np
lines = [l for l in open("gpurun_out/bprof.err") if l.startswith("ba_prof ")]
names = re.findall(r"([a-zA-Z]+) -?[0-9.]+", lines[0].split(":", 1)[1])
rows = [[float(v) for v in re.findall(r"(-?[0-9.]+)", l.split(":", 1)[1])] for l in lines]
a = np.median(np.array(rows[5:]), 0).round(1)
print("median us:", " ".join(f"{n}={v}" for n, v in zip(names, a) if v >= 0))
PY
RSPL_BA_TIMING=1 timeout -k 10 120 python -u tools/bench_ba.py --iters 20 > /dev/null 2> gpurun_out/btim.err || exit 1
python3 - <<'PY'
import re, numpy as np
rows = [[float(v) for v in re.findall(r" ([0-9.]+)", l.split(":", 1)[1])] for l in open("gpurun_out/btim.err") if l.startswith("rspl_ba_local us:")]
names = re.findall(r"([a-z0-9]+) [0-9.]+", [l for l in open("gpurun_out/btim.err") if l.startswith("rspl_ba_local")][0].split(":", 1)[1])
print("host stages median us:", " ".join(f"{n}={v}" for n, v in zip(names, np.median(np.array(rows[5:]), 0).round(0))))
PY
