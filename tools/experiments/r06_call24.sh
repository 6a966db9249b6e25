#!/bin/bash
# final tree check: full GPU suite, smoke, headline bench in the driver's shape
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/gpu_tests_final.log | head; tail -30 gpurun_out/gpu_tests_final.log; exit 1; }
tail -1 gpurun_out/gpu_tests_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke_final.log; exit 1; }
cat gpurun_out/smoke_final.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06_bench_final20.json 2> gpurun_out/bench20.err || { tail -20 gpurun_out/bench20.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('driver-shaped', d['value'], d['ms_per_step'], d['stages_ms_per_step']['ba:wall'])" gpurun_out/r06_bench_final20.json
