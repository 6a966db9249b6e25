#!/bin/bash
# dense reduced matrix (Sd) A/B: standalone C5 BA alternating base / Sd builds, then the in-kernel trace of each
set -o pipefail
mkdir -p gpurun_out
for lib in librspl_base.so librspl.so librspl_base.so librspl.so librspl_base.so librspl.so; do
  RSPL_LIB=$lib timeout -k 10 120 python -u tools/bench_ba.py --iters 10 --poses 30 --points 10000 --lines 0 2>&1 | tail -1 | sed "s/^/$lib: /" || exit 1
done
for lib in librspl_base.so librspl.so; do
RSPL_LIB=$lib RSPL_BA_PROF=1 timeout -k 10 120 python -u tools/bench_ba.py --iters 5 --poses 30 --points 10000 --lines 0 > /dev/null 2> gpurun_out/c5prof_$lib.err || exit 1
echo $lib; grep "ba_prof us" gpurun_out/c5prof_$lib.err | tail -2
done
