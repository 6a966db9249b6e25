#!/bin/bash
# Scratch GPU command of the current experiment (rewritten per experiment).
# A/B on one box: HEAD library (staging thread) vs the working tree (+ deferred copy-out at the seam
# between two tracking-thread calls), alternating headline benches.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3 4; do
  for lib in librspl_base.so librspl.so; do
    RSPL_LIB=$lib timeout -k 10 200 python3 bench.py --steps 300 --warmup 10 --no-cpu-baseline --single-precision > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench $lib failed"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], 'ba', s.get('ba:wall'), 'queue', d['host_ms_per_step']['ba_queue'])" gpurun_out/ab.json $lib
  done
done
