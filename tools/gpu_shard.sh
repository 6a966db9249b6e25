#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba_shard.py tests/test_gpu_ba.py tests/test_gpu_large.py -k "ba or group or rccl" -x -v --timeout 300 --timeout-method thread > gpurun_out/shard_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/shard_tests.log; exit 1; }
tail -25 gpurun_out/shard_tests.log
