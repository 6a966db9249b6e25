#!/bin/bash
R=$PWD
cd /tmp && export TMPDIR=/tmp
for cfg in "--lines 0" "--points 200 --lines 100" "--points 4000 --lines 100"; do
  n=$(echo $cfg | tr -d ' -')
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_split_$n -o run -- python3 $R/tools/bench_ba.py --iters 5 $cfg > /dev/null 2>&1 || exit 1
  echo "== $cfg"
  python3 $R/tools/prof_stats.py $R/gpurun_out/prof_split_$n/run_results.db | head -7 | cut -c1-160
done
