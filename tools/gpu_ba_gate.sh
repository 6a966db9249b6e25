#!/bin/bash
# BA parity tests, standalone BA timing (gated / ungated), the bench line and the BA timeline.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_ba_shard.py tests/test_gpu_large.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ba_tests.log; exit 1; }
tail -2 gpurun_out/ba_tests.log
timeout -k 10 300 python -u tools/bench_ba.py > gpurun_out/bench_ba.log 2>&1 || { echo "bench_ba failed"; tail -30 gpurun_out/bench_ba.log; exit 1; }
echo "gated:   $(tail -1 gpurun_out/bench_ba.log)"
RSPL_BA_UNGATED=1 timeout -k 10 300 python -u tools/bench_ba.py > gpurun_out/bench_ba_ug.log 2>&1 || { echo "bench_ba failed"; tail -30 gpurun_out/bench_ba_ug.log; exit 1; }
echo "ungated: $(tail -1 gpurun_out/bench_ba_ug.log)"
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-300 gpurun_out/bench.json
bash tools/gpu_ba_tl.sh | tail -14
