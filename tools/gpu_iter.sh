#!/bin/bash
# One development iteration on the GPU box: the GPU parity tests of the touched components, then
# the headline bench (short CPU-baseline-free run) and a standalone BA timing.
# usage: bash tools/gpu_iter.sh "<pytest file list>" [bench extra args]
set -o pipefail
mkdir -p gpurun_out
TESTS=${1:-tests}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/iter_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/iter_tests.log; exit 1; }
tail -3 gpurun_out/iter_tests.log
timeout -k 10 200 python -u tools/bench_ba.py --iters 30 > gpurun_out/iter_ba.log 2>&1 || { echo "bench_ba failed"; tail -20 gpurun_out/iter_ba.log; exit 1; }
cat gpurun_out/iter_ba.log
timeout -k 10 300 python -u bench.py --single-precision --no-cpu-baseline $2 > gpurun_out/iter_bench.json 2> gpurun_out/iter_bench.err || { echo "bench failed"; tail -30 gpurun_out/iter_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/iter_bench.json'))
print('value', d['value'], 'ms/step', d['ms_per_step'])
print('stages', d['stages_ms_per_step'])
print('roofline', d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
