#!/bin/bash
# BA record layout check: BA / map / shard parity tests, determinism repeats, standalone timing,
# per-kernel stats of the standalone C3 solve and the pipeline bench line.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_ba_shard.py tests/test_gpu_large.py tests/test_gpu_map.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ba_tests.log; exit 1; }
tail -2 gpurun_out/ba_tests.log
timeout -k 10 200 python -u tools/ba_repeat.py > gpurun_out/ba_repeat.log 2>&1 || { echo "repeat failed"; tail -20 gpurun_out/ba_repeat.log; exit 1; }
tail -4 gpurun_out/ba_repeat.log
timeout -k 10 60 python -u tools/bench_ba.py --iters 50 || exit 1
timeout -k 10 60 python -u tools/bench_ba.py --iters 10 --poses 30 --points 10000 --lines 0 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ba -o run -- python3 tools/bench_ba.py --iters 50 > gpurun_out/prof_ba.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_ba.log; exit 1; }
timeout -k 10 300 python -u bench.py --single-precision --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['ms_per_step'], d['ba'], d['stages_ms_per_step'])"
