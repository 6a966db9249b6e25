#!/bin/bash
# C3 headline A/B on one box: the morning's library (90bc551, before solve_reg / chunk_geo) vs HEAD, alternating
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for lib in librspl_base.so librspl.so; do
  RSPL_LIB=$lib timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/ab_$lib.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['stages_ms_per_step'].get('ba:wall'))" gpurun_out/ab_$lib.json $lib
done; done
