#!/bin/bash
# A/B of the reduced-system solvers (RSPL_BA_SOLVE = blk4 | wave | lds): BA GPU parity tests with the
# default, then per solver the standalone C3 BA time and the in-kernel trial trace (RSPL_BA_PROF).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_ba_shard.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for m in blk4 wave lds; do
  RSPL_BA_SOLVE=$m timeout -k 10 120 python -u tools/bench_ba.py --iters 30 > gpurun_out/ab_$m.log 2>&1 || { echo "bench $m failed"; tail -5 gpurun_out/ab_$m.log; exit 1; }
  echo "$m: $(cat gpurun_out/ab_$m.log)"
  RSPL_BA_SOLVE=$m RSPL_BA_PROF=1 timeout -k 10 120 python -u tools/bench_ba.py --iters 20 > /dev/null 2> gpurun_out/ab_prof_$m.err || exit 1
done
python3 - <<'PY'
import re, numpy as np
for m in ("blk4", "wave", "lds"):
    lines = [l for l in open(f"gpurun_out/ab_prof_{m}.err") if l.startswith("ba_prof ")]
    names = re.findall(r"([a-zA-Z]+) -?[0-9.]+", lines[0].split(":", 1)[1])
    rows = [[float(v) for v in re.findall(r"(-?[0-9.]+)", l.split(":", 1)[1])] for l in lines]
    a = np.median(np.array(rows[5:]), 0).round(1)
    print(m, "median us:", " ".join(f"{n}={v}" for n, v in zip(names, a)))
PY
