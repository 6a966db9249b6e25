#!/bin/bash
# Scratch GPU command of the current experiment (rewritten per experiment).
# BA register diet (pair_chunk 256 VGPRs) + tight line table + native tracking thread: GPU BA / map tests,
# then A/B/C: HEAD lib + Python thread, new lib + Python thread, new lib + native thread; host stage times.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_ba.py tests/test_gpu_map.py tests/test_gpu_ba_shard.py tests/test_gpu_large.py -k "ba or map" -x -q --timeout 120 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 || { echo "BA tests failed"; tail -30 gpurun_out/ba_tests.log; exit 1; }
tail -1 gpurun_out/ba_tests.log
for r in 1 2 3; do
  for v in "librspl_base.so python" "librspl.so python" "librspl.so native"; do
    set -- $v
    RSPL_LIB=$1 timeout -k 10 200 python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline --single-precision --ba-thread $2 > gpurun_out/bt.json 2> gpurun_out/bt.err || { echo "bench $v failed"; tail -5 gpurun_out/bt.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], 'ba', d['stages_ms_per_step'].get('ba:wall'), 'queue', d['host_ms_per_step']['ba_queue'])" gpurun_out/bt.json "$v"
  done
done
RSPL_BA_TIMING=1 timeout -k 10 200 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --single-precision > gpurun_out/btim.json 2> gpurun_out/btim.err || { echo "timing bench failed"; tail -5 gpurun_out/btim.err; exit 1; }
python3 - <<'PY'
import collections, numpy as np
d = collections.defaultdict(list)
for l in open('gpurun_out/btim.err'):
    if l.startswith('rspl_ba_local us:'):
        t = l.split()[3:]
        for k, v in zip(t[::2], t[1::2]): d[k].append(float(v))
print('host stage medians (us):', {k: round(float(np.median(v[len(v)//4:])), 1) for k, v in d.items()})
PY
timeout -k 10 120 python3 -u tools/bench_ba.py --iters 30 2>&1 | tail -3
