#!/bin/bash
# BA parity tests + BA timing + the default bench line (one GPU call, each step time-limited).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_ba_shard.py tests/test_gpu_large.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ba_tests.log; exit 1; }
tail -3 gpurun_out/ba_tests.log
timeout -k 10 300 python -u tools/bench_ba.py > gpurun_out/bench_ba.log 2>&1 || { echo "bench_ba failed"; tail -30 gpurun_out/bench_ba.log; exit 1; }
tail -5 gpurun_out/bench_ba.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
