#!/bin/bash
# A/B of two in-tree builds of librspl (RSPL_LIB=librspl_old.so vs the current librspl.so):
# standalone C3 / C5 local-BA timing and the pipeline bench, alternated.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for L in librspl_old.so librspl.so; do
    echo "== $L"
    RSPL_LIB=$L timeout -k 10 60 python -u tools/bench_ba.py --iters 50 || exit 1
    RSPL_LIB=$L timeout -k 10 60 python -u tools/bench_ba.py --iters 10 --poses 30 --points 10000 --lines 0 || exit 1
    RSPL_LIB=$L timeout -k 10 200 python -u bench.py --single-precision --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench failed"; tail -20 gpurun_out/ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); s=d['stages_ms_per_step']; print('bench', d['value'], 'ba', s['ba:wall'])"
  done
done
