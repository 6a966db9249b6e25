#!/bin/bash
# Scratch GPU command of the current experiment (rewritten per experiment).
# The call's final kernel queued behind optimize(5)'s trials (gated on the LM control's stop flag): BA GPU
# tests, standalone BA, then alternating headline benches HEAD vs the working tree.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ba.py tests/test_gpu_map.py tests/test_gpu_large.py tests/test_gpu_ba_shard.py -k "ba or map" -x -q --timeout 200 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 || { echo "BA tests failed"; tail -30 gpurun_out/ba_tests.log; exit 1; }
tail -1 gpurun_out/ba_tests.log
for lib in librspl_base.so librspl.so; do
  RSPL_LIB=$lib timeout -k 10 120 python -u tools/bench_ba.py --iters 30 || exit 1
done
for r in 1 2 3; do
  for lib in librspl_base.so librspl.so; do
    RSPL_LIB=$lib timeout -k 10 200 python3 bench.py --steps 300 --warmup 10 --no-cpu-baseline --single-precision > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench $lib failed"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], 'ba', s.get('ba:wall'))" gpurun_out/ab.json $lib
  done
done
