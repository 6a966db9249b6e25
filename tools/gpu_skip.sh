#!/bin/bash
# BA wall time in the bench loop with stages left out (diagnostics, not benchmark lines): which
# co-running stream slows the BA chain.
set -o pipefail
mkdir -p gpurun_out
for S in none sg sp sp,sg; do
  if [ $S = none ]; then A=""; else A="--skip $S"; fi
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision --steps 100 $A > gpurun_out/skip.json 2> gpurun_out/skip.err || { echo "bench $S failed"; tail -20 gpurun_out/skip.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/skip.json')); print(sys.argv[1], d['value'], 'ba', d['ba']['ms_per_call'] if 'ba' in d else d.get('stages_ms_per_step',{}).get('ba:wall'))" $S
done
