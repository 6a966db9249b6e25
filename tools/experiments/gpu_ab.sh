#!/bin/bash
# Alternating A/B of the headline bench under environment variants (same box, same tree).
# Usage: tools/experiments/gpu_ab.sh "A_ENV" "B_ENV" [rounds] [extra bench args]; each variant's line goes to
# gpurun_out/ab_<i>_<A|B>.json and a summary (frames/s, ba:wall, lines) is printed.
set -o pipefail
A="$1"; B="$2"; N=${3:-2}; shift 3 2>/dev/null; EXTRA="$*"
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for v in A B; do
    if [ $v = A ]; then E="$A"; else E="$B"; fi
    env $E timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision $EXTRA > gpurun_out/ab_${i}_${v}.json 2> gpurun_out/ab_${i}_${v}.err || { echo "bench $v failed"; tail -20 gpurun_out/ab_${i}_${v}.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_${i}_${v}.json').read().strip().splitlines()[-1]); s=d.get('stages_ms_per_step',{})
print('$v', '[$E]', round(d['value'],1), 'f/s', d['ms_per_step'], 'ms; ba', s.get('ba:wall'), 'gnn', s.get('sg:gnn x18'), 'sink', s.get('sg:sinkhorn'))"
  done
done
