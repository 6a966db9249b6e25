#!/bin/bash
# Full GPU suite (one pytest process), then smoke.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error" gpurun_out/gpu_tests.log | tail -5; tail -40 gpurun_out/gpu_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
