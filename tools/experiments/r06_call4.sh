#!/bin/bash
# Round-6 GPU call 4: FrameOptimization reading its inputs from the mapped staging; PnP refinement on four waves.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_pnp.py -x -v --timeout 200 --timeout-method thread > gpurun_out/fp_tests.log 2>&1 \
    || { tail -40 gpurun_out/fp_tests.log; exit 1; }
tail -3 gpurun_out/fp_tests.log
timeout -k 10 300 python -u tools/bench_frame.py > gpurun_out/r06_bench_frame.json 2> gpurun_out/bench_frame.err || { tail -20 gpurun_out/bench_frame.err; exit 1; }
cat gpurun_out/r06_bench_frame.json
