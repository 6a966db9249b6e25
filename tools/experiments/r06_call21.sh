#!/bin/bash
# PnP Jacobi on per-lane 2 x 2 blocks: PnP / frame GPU tests, bitwise A/B against the base build, in-kernel phases,
# bench alternating
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pnp.py tests/test_gpu_frame.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fp_tests.log 2>&1 \
    || { grep -E "FAILED|Error" gpurun_out/fp_tests.log | head -20; tail -30 gpurun_out/fp_tests.log; exit 1; }
tail -1 gpurun_out/fp_tests.log
RSPL_LIB=librspl_base.so timeout -k 10 120 python -u tools/experiments/frame_pnp_dump.py gpurun_out/fp_base.npz || exit 1
RSPL_LIB=librspl.so timeout -k 10 120 python -u tools/experiments/frame_pnp_dump.py gpurun_out/fp_new.npz || exit 1
python3 tools/experiments/frame_pnp_cmp.py gpurun_out/fp_base.npz gpurun_out/fp_new.npz
RSPL_PNP_PROF=1 timeout -k 10 200 python -u tools/bench_frame.py --batch 2 --iters 3 > /dev/null 2> gpurun_out/pprof.err || { tail -20 gpurun_out/pprof.err; exit 1; }
grep pnp_prof gpurun_out/pprof.err | head -3 || true
for lib in librspl_base.so librspl.so librspl_base.so librspl.so; do
  RSPL_LIB=$lib timeout -k 10 200 python -u tools/bench_frame.py > gpurun_out/bf_$lib.json 2> gpurun_out/bf.err || { tail -20 gpurun_out/bf.err; exit 1; }
  echo $lib; cat gpurun_out/bf_$lib.json
done
