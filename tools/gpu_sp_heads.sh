#!/bin/bash
# SuperPoint fp16 heads: SP parity tests (fp32 exact path and the fp16 bar), the SP+SG pipeline
# tests, then the bench line with per-stage times.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sp.py tests/test_gpu_large.py tests/test_abi_c.py -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/sp_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/sp_tests.log; exit 1; }
grep -E "overlap|passed|failed" gpurun_out/sp_tests.log | tail -6
timeout -k 10 300 python -u bench.py --single-precision --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['ms_per_step'], d['stages_ms_per_step'])"
