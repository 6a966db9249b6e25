#!/bin/bash
# Scratch GPU command of the current experiment (rewritten per experiment).
# C5 LDS solve: in-kernel trace (assembly, factor, back-substitution; first two steps' panel / trailing
# update) for HEAD vs the working tree.
set -o pipefail
mkdir -p gpurun_out
for lib in librspl_base.so librspl.so; do
  RSPL_LIB=$lib RSPL_BA_PROF=1 timeout -k 10 120 python -u tools/bench_ba.py --iters 6 --poses 30 --points 10000 --lines 0 > /dev/null 2> gpurun_out/bprof.err || exit 1
  LIB=$lib python3 - <<'PY'
import os, re, numpy as np
lines = [l for l in open("gpurun_out/bprof.err") if l.startswith("ba_prof ")]
names = re.findall(r"([a-zA-Z]+) -?[0-9.]+", lines[0].split(":", 1)[1])
rows = [[float(v) for v in re.findall(r"(-?[0-9.]+)", l.split(":", 1)[1])] for l in lines]
a = np.median(np.array(rows[2:]), 0).round(1)
print(os.environ['LIB'], "median us:", " ".join(f"{n}={v}" for n, v in zip(names, a) if v >= 0))
PY
done
