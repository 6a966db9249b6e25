#!/bin/bash
# 28-value all-reduce on permlane swaps + fused block combine: frame / PnP GPU tests, bitwise A/B against the base
# build, per-phase cycles (librspl_fprof.so), frame / PnP bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_pnp.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fp_tests.log 2>&1 \
    || { grep -E "FAILED|Error" gpurun_out/fp_tests.log | head -20; tail -30 gpurun_out/fp_tests.log; exit 1; }
tail -1 gpurun_out/fp_tests.log
RSPL_LIB=librspl_base.so timeout -k 10 120 python -u tools/experiments/frame_pnp_dump.py gpurun_out/fp_base.npz || exit 1
RSPL_LIB=librspl.so timeout -k 10 120 python -u tools/experiments/frame_pnp_dump.py gpurun_out/fp_new.npz || exit 1
python3 tools/experiments/frame_pnp_cmp.py gpurun_out/fp_base.npz gpurun_out/fp_new.npz
RSPL_LIB=librspl_fprof.so timeout -k 10 200 python -u tools/bench_frame.py --batch 2 --iters 3 > gpurun_out/fprof.json 2> gpurun_out/fprof.err || { tail -20 gpurun_out/fprof.err; exit 1; }
grep fprof gpurun_out/fprof.err | head -3 || true
for lib in librspl_base.so librspl.so librspl_base.so librspl.so; do
  RSPL_LIB=$lib timeout -k 10 200 python -u tools/bench_frame.py > gpurun_out/bf_$lib.json 2> gpurun_out/bf.err || { tail -20 gpurun_out/bf.err; exit 1; }
  echo $lib; cat gpurun_out/bf_$lib.json
done
