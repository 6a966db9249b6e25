#!/bin/bash
# Round-6 A/B: BA waves at issue priority 3 (librspl.so) vs the plain priority (librspl_base.so), alternating,
# the driver's bench shape (20 / 5) and 200 steps; then the BA alone.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for L in librspl_base.so librspl.so; do
    RSPL_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --single-precision --no-cpu-baseline \
        > gpurun_out/ab_$L.$i.json 2> gpurun_out/ab_$L.$i.err || { tail -5 gpurun_out/ab_$L.$i.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open('gpurun_out/ab_$L.$i.json'));print('$L 20/5', d['value'], d['stages_ms_per_step']['ba:wall'])"
  done
done
for L in librspl_base.so librspl.so; do
  RSPL_LIB=$L timeout -k 10 300 python -u bench.py --single-precision --no-cpu-baseline > gpurun_out/ab200_$L.json 2> gpurun_out/ab200_$L.err \
      || { tail -5 gpurun_out/ab200_$L.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab200_$L.json'));print('$L 200', d['value'], d['stages_ms_per_step']['ba:wall'], d['stages_ms_per_step']['sg:gnn x18'], d['stages_ms_per_step']['sp:conv1a+1b+pool'])"
done
