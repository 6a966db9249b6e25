#!/bin/bash
# Sinkhorn exchange rework: SG / NMS parity tests, then per-G timing of the SG call (2 pairs, N=400)
# and the in-kernel phase probe.  Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sg.py tests/test_gpu_sp.py tests/test_gpu_large.py -m gpu -x -v -s --timeout 200 --timeout-method thread -k "sg or nms or sinkhorn or decode" > gpurun_out/sink_tests.log 2>&1 || { echo "tests failed"; grep -E "max \|dZ\||PASS|FAIL|Error|error" gpurun_out/sink_tests.log | tail -40; exit 1; }
grep -E "max \|dZ\||passed|failed" gpurun_out/sink_tests.log
for G in ${SINK_GS:-16 24 32}; do
  RSPL_SG_SINK_G=$G timeout -k 10 60 python -u tools/bench_sg.py --precision fp16 --iters 100 || exit 1
  RSPL_SG_SINK_G=$G RSPL_SG_PROBE=1 timeout -k 10 60 python -u tools/bench_sg.py --precision fp16 --iters 2 2>&1 | tail -2 || exit 1
done
