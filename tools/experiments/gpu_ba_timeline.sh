#!/bin/bash
# Kernel timeline of standalone C3 BA calls (rocprofv3 kernel trace): per-dispatch start / gap / duration
# of the last call, to see where a call's wall time goes outside the LM trials.  BA_ARGS: extra
# tools/bench_ba.py arguments (e.g. the C5 shape: --poses 30 --points 10000 --lines 0).
set -o pipefail
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_ba -o run -- python3 $R/tools/bench_ba.py --iters 4 ${BA_ARGS} > $R/gpurun_out/prof_ba.log 2>&1 || { tail -20 $R/gpurun_out/prof_ba.log; exit 1; }
cd $R
python3 tools/prof_timeline.py $(find gpurun_out/prof_ba -name '*results.db' | head -1) ${NTAIL:-45} > gpurun_out/ba_timeline.txt || exit 1
rm -rf gpurun_out/prof_ba
cat gpurun_out/ba_timeline.txt
