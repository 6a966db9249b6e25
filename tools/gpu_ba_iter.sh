#!/bin/bash
# BA parity tests, then the in-kernel trial spans (alone / in the pipeline) and the bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_ba_shard.py tests/test_gpu_large.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ba_tests.log; exit 1; }
tail -2 gpurun_out/ba_tests.log
bash tools/gpu_baprof.sh || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-400 gpurun_out/bench.json
