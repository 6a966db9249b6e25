#!/bin/bash
# Round-6 GPU call 6: same-box A/B of the native map's parallel passes (librspl_base.so = the sequential map),
# alternating, GPU path only.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for L in librspl_base.so librspl.so; do
    RSPL_LIB=$L timeout -k 10 200 python -u tools/run_sequence.py --no-cpu --out gpurun_out/seq_ab > gpurun_out/seq_ab_$L.$i.json 2>/dev/null || exit 1
    echo "$L $(cat gpurun_out/seq_ab_$L.$i.json)"
  done
done
