#!/bin/bash
# FrameOptimization per-phase cycles (experiment build librspl_fprof.so, -DRSPL_FRAME_PROF): one 400-edge frame
set -o pipefail
mkdir -p gpurun_out
RSPL_LIB=librspl_fprof.so timeout -k 10 200 python -u tools/bench_frame.py --batch 2 --iters 3 > gpurun_out/fprof.json 2> gpurun_out/fprof.err || { tail -20 gpurun_out/fprof.err; exit 1; }
grep fprof gpurun_out/fprof.err | sort | uniq -c | head -20 || true
grep -h fprof gpurun_out/fprof.json | head -5 || true
cat gpurun_out/fprof.json | tail -3
