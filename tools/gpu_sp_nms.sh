#!/bin/bash
# SuperPoint tests (NMS units, EuRoC reference maps, large frames) + a rocprofv3 kernel trace of
# the fp16 bench step: per-kernel averages of the SP kernels
set -o pipefail
R=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sp.py tests/test_gpu_large.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sp_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/sp_tests.log; exit 1; }
tail -2 gpurun_out/sp_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sp -o run -- python3 $R/bench.py --no-cpu-baseline --single-precision --steps 20 --warmup 5 > $R/gpurun_out/bench_sp.json 2> $R/gpurun_out/bench_sp.err || { echo "prof failed"; tail -20 $R/gpurun_out/bench_sp.err; exit 1; }
cd $R
python3 tools/prof_stats.py gpurun_out/prof_sp/run_results.db > gpurun_out/sp_kernel_stats.csv
grep -E "nms|topk|conv3x3_h_kernel<64|det_head|sample_taps" gpurun_out/sp_kernel_stats.csv | cut -c1-160
