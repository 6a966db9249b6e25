#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 200 python -u tools/bench_frame.py > gpurun_out/bench_frame.json 2> gpurun_out/bench_frame.err || { echo "bench_frame failed"; tail -20 gpurun_out/bench_frame.err; exit 1; }
cat gpurun_out/bench_frame.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_frame -o run -- python3 $R/tools/bench_frame.py --iters 5 > /dev/null 2>&1 || { echo "prof failed"; exit 1; }
python3 $R/tools/prof_stats.py $R/gpurun_out/prof_frame/run_results.db | head -5
