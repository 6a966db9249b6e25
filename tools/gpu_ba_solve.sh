#!/bin/bash
# Reduced-system solve A/B: BA parity tests, repeatability, standalone timing and in-kernel trial
# spans with the register-tiled small solve vs the packed-LDS kernel (RSPL_BA_SOLVE_PACKED=1).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_ba_shard.py tests/test_gpu_map.py tests/test_gpu_large.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ba_tests.log; exit 1; }
tail -1 gpurun_out/ba_tests.log
timeout -k 10 120 python -u tools/ba_repeat.py || exit 1
for M in packed small; do
  if [ $M = packed ]; then export RSPL_BA_SOLVE_PACKED=1; else unset RSPL_BA_SOLVE_PACKED; fi
  echo "== $M"
  timeout -k 10 60 python -u tools/bench_ba.py --iters 50 || exit 1
  RSPL_BA_PROF=1 timeout -k 10 100 python -u tools/bench_ba.py --iters 20 2> gpurun_out/bp_$M.err > /dev/null || exit 1
  python3 - "$M" <<'PY'
import re, sys, numpy as np
lines = [l for l in open(f"gpurun_out/bp_{sys.argv[1]}.err") if l.startswith("ba_prof ")]
names = re.findall(r"([a-z]+) -?[0-9.]+", lines[0].split(":", 1)[1])
rows = [[float(v) for v in re.findall(r"(-?[0-9.]+)", l.split(":", 1)[1])] for l in lines]
a = np.median(np.array(rows[5:]), 0).round(1)
print("median us:", " ".join(f"{n}={v}" for n, v in zip(names, a)))
PY
done
