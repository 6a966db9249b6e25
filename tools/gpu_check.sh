#!/bin/bash
# One GPU call: parity tests, smoke, bench, rocprof kernel stats.  Each GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --no-cpu-baseline --single-precision > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || { echo "prof failed"; tail -30 $R/gpurun_out/prof_bench.err; exit 1; }
cat $R/gpurun_out/prof_bench.json
