#!/bin/bash
# Session-2 baseline on the restored tree: GPU tests, smoke, headline bench (200 steps), driver shape, 100-keyframe
# map sequence (assembly cost after the map.cpp rewrite).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
    || { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/s2_bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['ms_per_step'], d['stages_ms_per_step'].get('ba:wall'))" gpurun_out/s2_bench.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s2_bench20.json 2> gpurun_out/bench20.err || { tail -30 gpurun_out/bench20.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('driver-shaped', d['value'], d['ms_per_step'])" gpurun_out/s2_bench20.json
timeout -k 10 500 python -u tools/run_sequence.py --out gpurun_out/s2_sequence > gpurun_out/s2_sequence100.json 2> gpurun_out/seq.err || { tail -5 gpurun_out/seq.err; exit 1; }
cat gpurun_out/s2_sequence100.json
