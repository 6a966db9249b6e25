#!/bin/bash
# Round-6 GPU call 7: the full GPU suite + smoke after the knob pruning, then the headline bench (20 / 5, the
# driver's shape) and the default 200-step run.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
    || { grep -E "FAILED|Error|error" gpurun_out/gpu_tests.log | head -20; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench20.json 2> gpurun_out/bench20.err || { tail -20 gpurun_out/bench20.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench20.json'));print('20/5', d['value'], d.get('fp16x3_run',{}).get('value'), d['stages_ms_per_step']['ba:wall'])"
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench200.json 2> gpurun_out/bench200.err || { tail -20 gpurun_out/bench200.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench200.json'));print('200', d['value'], d.get('fp16x3_run',{}).get('value'), d['stages_ms_per_step']['ba:wall'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline'].get('mfma_busy'))"
