#!/bin/bash
# dense reduced matrix (Sd) written by the pair-completing Schur chunks, read by solve_reg's tile init: BA / C5 /
# shard / map GPU tests, C5 BA micro-bench and C5 bench twice
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_large.py tests/test_gpu_ba_shard.py tests/test_gpu_map.py tests/test_abi_c.py -x -v --timeout 300 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 \
    || { grep -E "FAILED|Error" gpurun_out/ba_tests.log | head -20; tail -30 gpurun_out/ba_tests.log; exit 1; }
tail -1 gpurun_out/ba_tests.log
timeout -k 10 120 python -u tools/bench_ba.py --iters 10 --poses 30 --points 10000 --lines 0 2>&1 | tail -1 || exit 1
timeout -k 10 120 python -u tools/bench_ba.py --iters 30 2>&1 | tail -1 || exit 1
for r in 1 2; do
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline --single-precision > gpurun_out/r06_bench_c5_sd$r.json 2> gpurun_out/c5.err || { tail -5 gpurun_out/c5.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c5', d['value'], d['ms_per_step'], d['stages_ms_per_step'].get('ba:wall'))" gpurun_out/r06_bench_c5_sd$r.json
done
