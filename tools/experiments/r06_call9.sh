#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_pnp.py -x -v --timeout 200 --timeout-method thread > gpurun_out/fp_tests.log 2>&1 \
    || { grep -E "FAILED|Error" gpurun_out/fp_tests.log | head; tail -40 gpurun_out/fp_tests.log; exit 1; }
tail -1 gpurun_out/fp_tests.log
ROUND=r06 bash tools/gpu_round_side.sh
