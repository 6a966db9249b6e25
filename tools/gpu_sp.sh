#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sp.py tests/test_gpu_large.py -k "sp or SP or fp16" -x -v --timeout 200 --timeout-method thread > gpurun_out/sp_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/sp_tests.log; exit 1; }
grep -E "PASS|FAIL|fp16 SP|overlap" gpurun_out/sp_tests.log | tail -20
timeout -k 10 300 python -u bench.py --no-cpu-baseline --single-precision --steps 30 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo "bench failed"; tail -20 gpurun_out/bench_quick.err; exit 1; }
cat gpurun_out/bench_quick.json
