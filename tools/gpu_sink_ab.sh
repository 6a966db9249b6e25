#!/bin/bash
# Alternating A/B of Sinkhorn workgroups per pair in the pipeline (frames/s, Sinkhorn, BA wall).
set -o pipefail
export RSPL_SG_SINK=slab  # these sweeps are of the slab kernel (RSPL_SG_SINK_G); the row-block kernel is the default
mkdir -p gpurun_out
for rep in 1 2 3; do
  for G in 32 48; do
    RSPL_SG_SINK_G=$G timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision --steps 200 > gpurun_out/sg_g.json 2> gpurun_out/sg_g.err || { echo "bench failed"; tail -20 gpurun_out/sg_g.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/sg_g.json')); s=d['stages_ms_per_step']; print('G', sys.argv[1], d['value'], 'sink', s['sg:sinkhorn'], 'ba', s['ba:wall'])" $G
  done
done
