#!/bin/bash
# Round-6 GPU call 5: native map with parallel passes -- map GPU tests, the 100-keyframe sequence (numeric and
# analytic line Jacobian), FrameOptimization single-frame kernel trace.
set -o pipefail
R=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_map.py -x -v --timeout 300 --timeout-method thread > gpurun_out/map_tests.log 2>&1 \
    || { tail -40 gpurun_out/map_tests.log; exit 1; }
tail -3 gpurun_out/map_tests.log
timeout -k 10 400 python -u tools/run_sequence.py --out gpurun_out/seq_num > gpurun_out/r06_sequence100.json 2> gpurun_out/seq_num.err \
    || { tail -5 gpurun_out/seq_num.err; exit 1; }
cat gpurun_out/r06_sequence100.json
timeout -k 10 400 python -u tools/run_sequence.py --analytic-line-jacobian --out gpurun_out/seq_analytic \
    > gpurun_out/r06_sequence100_analytic.json 2> gpurun_out/seq_analytic.err || { tail -5 gpurun_out/seq_analytic.err; exit 1; }
cat gpurun_out/r06_sequence100_analytic.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_frame -o run -- python3 $R/tools/bench_frame.py --batch 1024 \
    > $R/gpurun_out/prof_frame.txt 2>&1 || { tail -5 $R/gpurun_out/prof_frame.txt; exit 1; }
cd $R
python3 tools/prof_stats.py gpurun_out/prof_frame/run_results.db > gpurun_out/r06_frame_kernel_stats.csv && rm -rf gpurun_out/prof_frame
head -8 gpurun_out/r06_frame_kernel_stats.csv | cut -c1-150
