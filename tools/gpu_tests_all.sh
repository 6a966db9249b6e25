#!/bin/bash
# All GPU tests without stopping at the first failure (each test bounded by its own timeout), then smoke.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
exit $rc
