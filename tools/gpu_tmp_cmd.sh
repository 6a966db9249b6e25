#!/bin/bash
# Scratch GPU command of the current experiment (rewritten per experiment).
# update_errors: each lane's second edge loaded with its first (no dependent round trips in the
# back-substitution / cost loops for landmarks with 9..16 edges).  BA GPU tests, standalone BA time and
# trial trace for HEAD vs the working tree, then alternating headline benches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ba.py tests/test_gpu_map.py tests/test_gpu_large.py -k "ba or map" -x -q --timeout 120 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 || { echo "BA tests failed"; tail -30 gpurun_out/ba_tests.log; exit 1; }
tail -1 gpurun_out/ba_tests.log
for lib in librspl_base.so librspl.so; do
  RSPL_LIB=$lib timeout -k 10 120 python -u tools/bench_ba.py --iters 30 || exit 1
  RSPL_LIB=$lib RSPL_BA_PROF=1 timeout -k 10 120 python -u tools/bench_ba.py --iters 20 > /dev/null 2> gpurun_out/bprof.err || exit 1
  LIB=$lib python3 - <<'PY'
import os, re, numpy as np
lines = [l for l in open("gpurun_out/bprof.err") if l.startswith("ba_prof ")]
names = re.findall(r"([a-zA-Z]+) -?[0-9.]+", lines[0].split(":", 1)[1])
rows = [[float(v) for v in re.findall(r"(-?[0-9.]+)", l.split(":", 1)[1])] for l in lines]
a = np.median(np.array(rows[5:]), 0).round(1)
print(os.environ['LIB'], "median us:", " ".join(f"{n}={v}" for n, v in zip(names, a) if v >= 0))
PY
done
for r in 1 2 3; do
  for lib in librspl_base.so librspl.so; do
    RSPL_LIB=$lib timeout -k 10 200 python3 bench.py --steps 300 --warmup 10 --no-cpu-baseline --single-precision > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench $lib failed"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], 'ba', s.get('ba:wall'))" gpurun_out/ab.json $lib
  done
done
