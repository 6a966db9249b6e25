#!/bin/bash
# rocprofv3 kernel trace of standalone C3 BA calls: the last call's kernel timeline (durations, gaps).
set -o pipefail
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/ba_tl -o run -- python3 $R/tools/bench_ba.py --iters 5 > $R/gpurun_out/ba_tl.out 2>&1 || { tail -20 $R/gpurun_out/ba_tl.out; exit 1; }
cd $R
DB=$(find gpurun_out/ba_tl -name '*.db' | head -1)
python3 tools/prof_timeline.py $DB ${NK:-60} > gpurun_out/ba_tl.txt
cat gpurun_out/ba_tl.txt
