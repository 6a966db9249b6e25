#!/bin/bash
# FrameOptimization on 8 waves for frames of > 256 edges (librspl_nw8.so): frame tests on it, result drift against
# the 4-wave build, per-phase cycles, bench alternating; PnP in-kernel phases (RSPL_PNP_PROF)
set -o pipefail
mkdir -p gpurun_out
RSPL_LIB=librspl_nw8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_frame.py -x -q --timeout 200 --timeout-method thread > gpurun_out/f8_tests.log 2>&1 \
    || { grep -E "FAILED|Error" gpurun_out/f8_tests.log | head -20; tail -30 gpurun_out/f8_tests.log; exit 1; }
tail -1 gpurun_out/f8_tests.log
RSPL_LIB=librspl.so timeout -k 10 120 python -u tools/experiments/frame_pnp_dump.py gpurun_out/fp_new.npz || exit 1
RSPL_LIB=librspl_nw8.so timeout -k 10 120 python -u tools/experiments/frame_pnp_dump.py gpurun_out/fp_nw8.npz || exit 1
python3 tools/experiments/frame_pnp_cmp.py gpurun_out/fp_new.npz gpurun_out/fp_nw8.npz
RSPL_LIB=librspl_fprof.so timeout -k 10 200 python -u tools/bench_frame.py --batch 2 --iters 3 > gpurun_out/fprof.json 2> gpurun_out/fprof.err || { tail -20 gpurun_out/fprof.err; exit 1; }
grep fprof gpurun_out/fprof.json | head -3 || true
for lib in librspl.so librspl_nw8.so librspl.so librspl_nw8.so; do
  RSPL_LIB=$lib timeout -k 10 200 python -u tools/bench_frame.py > gpurun_out/bf_$lib.json 2> gpurun_out/bf.err || { tail -20 gpurun_out/bf.err; exit 1; }
  echo $lib; cat gpurun_out/bf_$lib.json
done
RSPL_PNP_PROF=1 timeout -k 10 200 python -u tools/bench_frame.py --batch 2 --iters 3 > /dev/null 2> gpurun_out/pprof.err || { tail -20 gpurun_out/pprof.err; exit 1; }
grep pnp_prof gpurun_out/pprof.err | head -4 || true
