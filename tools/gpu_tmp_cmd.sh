#!/bin/bash
# Scratch GPU command of the current experiment (rewritten per experiment).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_ba_shard.py tests/test_gpu_map.py tests/test_gpu_large.py -k "ba or map" -q --timeout 120 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 || { echo "BA tests failed"; tail -30 gpurun_out/ba_tests.log; exit 1; }
tail -1 gpurun_out/ba_tests.log
for lib in librspl_base.so librspl.so librspl_base.so librspl.so; do
  RSPL_LIB=$lib RSPL_BA_TIMING=1 timeout -k 10 120 python -u tools/bench_ba.py --iters 30 2> gpurun_out/btim.err || exit 1
  grep rspl_ba_local gpurun_out/btim.err | tail -1
  RSPL_LIB=$lib timeout -k 10 120 python -u tools/bench_ba.py --iters 8 --poses 30 --points 10000 --lines 0 || exit 1
done
BA_ARGS="--poses 30 --points 10000 --lines 0" NTAIL=40 bash tools/gpu_ba_timeline.sh | head -60
