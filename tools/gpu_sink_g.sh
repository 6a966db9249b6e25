#!/bin/bash
# Sinkhorn workgroups per pair: standalone SuperGlue stage times and the pipeline line per G.
set -o pipefail
export RSPL_SG_SINK=slab  # these sweeps are of the slab kernel (RSPL_SG_SINK_G); the row-block kernel is the default
mkdir -p gpurun_out
for G in 32 48 64 100; do
  RSPL_SG_SINK_G=$G timeout -k 10 120 python -u tools/bench_sg.py --iters 30 2>&1 | tail -1 | sed "s/^/G=$G /" || exit 1
done
for G in 32 64; do
  RSPL_SG_SINK_G=$G timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision --steps 100 > gpurun_out/sg_g.json 2> gpurun_out/sg_g.err || { echo "bench failed"; tail -20 gpurun_out/sg_g.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sg_g.json')); s=d['stages_ms_per_step']; print('G', sys.argv[1], d['value'], 'sink', s['sg:sinkhorn'], 'ba', s['ba:wall'])" $G
done
