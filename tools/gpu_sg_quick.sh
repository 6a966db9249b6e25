#!/bin/bash
# SuperGlue parity (fp32 + fp16, printing the fp16 agreement) and the SG-only timing.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sg.py tests/test_gpu_large.py -k "sg or SG" -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/sg_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/sg_tests.log; exit 1; }
grep -E "agreement|passed|failed" gpurun_out/sg_tests.log
timeout -k 10 300 python -u tools/bench_sg.py --precision fp16 > gpurun_out/bench_sg.log 2>&1 || { echo "bench_sg failed"; tail -30 gpurun_out/bench_sg.log; exit 1; }
cat gpurun_out/bench_sg.log
RSPL_SG_GEMM_LDS=1 timeout -k 10 300 python -u tools/bench_sg.py --precision fp16 > gpurun_out/bench_sg_lds.log 2>&1 || { echo "bench_sg lds failed"; tail -30 gpurun_out/bench_sg_lds.log; exit 1; }
cat gpurun_out/bench_sg_lds.log
