#!/bin/bash
# BA kernel stats + the timeline of the last BA call (bench_ba.py, C3 size).
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_batl -o run -- python3 $R/tools/bench_ba.py --iters 5 > /dev/null 2>&1 || exit 1
python3 $R/tools/prof_timeline.py $R/gpurun_out/prof_batl/run_results.db 90 > $R/gpurun_out/batl.txt
cat $R/gpurun_out/batl.txt | head -30
