#!/bin/bash
# Round-6 GPU call 2: split-fp16 SuperPoint -- SP GPU tests, standalone SP timing (fp16 vs fp16x3), and the
# headline bench with fp16x3 (second measurement: fp16).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/sp_tests.log 2>&1 \
    || { tail -40 gpurun_out/sp_tests.log; exit 1; }
tail -3 gpurun_out/sp_tests.log
for p in fp16 fp16x3; do
  timeout -k 10 120 python -u tools/bench_sp.py --precision $p > gpurun_out/bench_sp_$p.txt 2>&1 || { cat gpurun_out/bench_sp_$p.txt; exit 1; }
  cat gpurun_out/bench_sp_$p.txt
done
timeout -k 10 400 python -u bench.py --precision fp16x3 --no-cpu-baseline > gpurun_out/bench_x3.json 2> gpurun_out/bench_x3.err \
    || { tail -20 gpurun_out/bench_x3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_x3.json'));print(d['value'], d['fp16_run'], d['stages_ms_per_step'])"
