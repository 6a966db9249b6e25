#!/bin/bash
# BA library A/B on one box: the BA GPU tests on the default build, then C3 BA timing (tools/bench_ba.py)
# and the in-kernel trial trace (RSPL_BA_PROF) of each in-tree build named in $LIBS (RSPL_LIB), then the
# headline bench alternated between the first two builds.  Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
LIBS=${LIBS:-"librspl_r03.so librspl.so"}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_ba_shard.py tests/test_gpu_map.py tests/test_gpu_large.py -k "ba or map" -x -q --timeout 120 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 || { echo "BA tests failed"; tail -40 gpurun_out/ba_tests.log; exit 1; }
tail -2 gpurun_out/ba_tests.log
fi
for lib in $LIBS; do
  echo "== $lib"
  RSPL_LIB=$lib timeout -k 10 120 python -u tools/bench_ba.py --iters 30 || exit 1
  RSPL_LIB=$lib RSPL_BA_PROF=1 timeout -k 10 120 python -u tools/bench_ba.py --iters 20 > /dev/null 2> gpurun_out/bprof_$lib.err || exit 1
  python3 - gpurun_out/bprof_$lib.err <<'PY'
import re, sys, numpy as np
lines = [l for l in open(sys.argv[1]) if l.startswith("ba_prof ")]
names = re.findall(r"([a-zA-Z]+) -?[0-9.]+", lines[0].split(":", 1)[1])
rows = [[float(v) for v in re.findall(r"(-?[0-9.]+)", l.split(":", 1)[1])] for l in lines]
a = np.median(np.array(rows[5:]), 0).round(1)
print("median us:", " ".join(f"{n}={v}" for n, v in zip(names, a) if v >= 0))
cl = [l for l in open(sys.argv[1]) if l.startswith("ba_chunks")]
if cl:
    names = re.findall(r"([a-z]+[0-9]*) -?[0-9.]+", cl[0].split(":", 1)[1])
    ch = np.array([[float(v) for v in re.findall(r" (-?[0-9.]+)", l.split(":", 1)[1])] for l in cl])
    print("chunks us:", " ".join(f"{n}={v}" for n, v in zip(names, np.median(ch[5:] if len(ch) > 5 else ch, 0).round(1))))
PY
done
if [ -n "$BENCH_AB" ]; then
  set -- $LIBS
  bash tools/experiments/gpu_ab.sh "RSPL_LIB=$1" "RSPL_LIB=$2" ${BENCH_AB} || exit 1
fi
