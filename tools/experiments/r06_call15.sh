#!/bin/bash
# C5: front-end streams CU-masked off N CUs (the BA's 768-thread / 162 KB-LDS solve needs a whole free CU), alternating
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for rc in 0 8 16 32; do
  timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline --single-precision --reserve-cus $rc > gpurun_out/c5_rc$rc.json 2> gpurun_out/c5.err || { tail -5 gpurun_out/c5.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_ms_per_step']; print('reserve', sys.argv[2], d['value'], d['ms_per_step'], s.get('ba:wall'), s.get('sg:gnn x18'))" gpurun_out/c5_rc$rc.json $rc
done; done
