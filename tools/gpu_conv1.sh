#!/bin/bash
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_sp.py tests/test_gpu_large.py -k "sp or SP or fp16" -x -q --timeout 200 --timeout-method thread > gpurun_out/sp_tests.log 2>&1 || { tail -30 gpurun_out/sp_tests.log; exit 1; }
tail -2 gpurun_out/sp_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c1 -o run -- python3 $R/tools/bench_sp.py --iters 20 > $R/gpurun_out/c1.txt 2>&1 || exit 1
grep SP $R/gpurun_out/c1.txt
python3 $R/tools/prof_stats.py $R/gpurun_out/prof_c1/run_results.db | cut -c1-150 | head -12
