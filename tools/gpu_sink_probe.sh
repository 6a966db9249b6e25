#!/bin/bash
# Sinkhorn: SG parity tests, then per-phase probe at several workgroups-per-pair counts (SG alone, 2 pairs, N=400).
set -o pipefail
export RSPL_SG_SINK=slab  # these sweeps are of the slab kernel (RSPL_SG_SINK_G); the row-block kernel is the default
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sg.py tests/test_gpu_large.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sink_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/sink_tests.log; exit 1; }
tail -2 gpurun_out/sink_tests.log
for G in ${SINK_GS:-16 24 32}; do
  RSPL_SG_SINK_G=$G timeout -k 10 60 python -u tools/bench_sg.py --precision fp16 --iters 100 || exit 1
  RSPL_SG_SINK_G=$G RSPL_SG_PROBE=1 timeout -k 10 60 python -u tools/bench_sg.py --precision fp16 --iters 2 2>&1 | tail -2 || exit 1
done
