#!/bin/bash
# Scratch GPU command of the current experiment (rewritten per experiment).
# SP conv workgroups capped at one per CU (RSPL_SP_LDS_PAD: unused dynamic LDS) so a BA wave fits beside a
# conv wave on every SIMD: 0 (default) vs 8192 (conv1 only: 76 + 8 KB) vs 24576 (every conv layer).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for pad in 0 8192 24576; do
    RSPL_SP_LDS_PAD=$pad timeout -k 10 200 python3 bench.py --steps 300 --warmup 10 --no-cpu-baseline --single-precision > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench $pad failed"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); s=d['stages_ms_per_step']; print('pad', sys.argv[2], d['value'], d['ms_per_step'], 'ba', s.get('ba:wall'), 'conv1', s.get('sp:conv1a+1b+pool'), 'conv2-4', s.get('sp:conv2a..conv4b'), 'gnn', s.get('sg:gnn x18'))" gpurun_out/ab.json $pad
  done
done
