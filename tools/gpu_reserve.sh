#!/bin/bash
# CU reservation sweep: SP / SG / post streams CU-masked off R CUs (and the BA optionally confined to
# them): frames/s and BA wall per setting.
set -o pipefail
mkdir -p gpurun_out
for R in 0 16 32 64; do
  for OWN in 1 0; do
    if [ $R = 0 ] && [ $OWN = 0 ]; then continue; fi
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision --steps 100 --reserve-cus $R --ba-own-cus $OWN > gpurun_out/rs.json 2> gpurun_out/rs.err || { echo "bench R=$R failed"; tail -20 gpurun_out/rs.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/rs.json')); print(sys.argv[1:], d['value'], 'ba', d['ba']['ms_per_call'])" R=$R own=$OWN
  done
done
