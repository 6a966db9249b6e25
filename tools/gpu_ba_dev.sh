#!/bin/bash
# Device-side LM: BA parity tests, then C3 / C5 standalone timing with host- vs device-decided trials,
# the per-phase host timing, and the full bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_ba_shard.py tests/test_gpu_large.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ba_tests.log; exit 1; }
tail -2 gpurun_out/ba_tests.log
for M in host dev; do
  if [ $M = host ]; then export RSPL_BA_HOSTLM=1; else unset RSPL_BA_HOSTLM; fi
  echo "== $M"
  timeout -k 10 60 python -u tools/bench_ba.py --iters 50 || exit 1
  timeout -k 10 60 python -u tools/bench_ba.py --iters 10 --poses 30 --points 10000 --lines 0 || exit 1
  RSPL_BA_TIMING=1 timeout -k 10 60 python -u tools/bench_ba.py --iters 3 2>&1 | tail -2 || exit 1
done
unset RSPL_BA_HOSTLM
timeout -k 10 300 python -u bench.py --single-precision --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['ms_per_step'], d['ba'], d['stages_ms_per_step'])"
