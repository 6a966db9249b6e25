#!/bin/bash
# C5 Schur chunk split (diagonal pose pairs in sub-chunks) and earlier solver swap: BA GPU tests, C5 parity,
# standalone C5 BA A/B against the previous library, C5 bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_large.py tests/test_gpu_ba_shard.py tests/test_gpu_map.py -x -v --timeout 300 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 \
    || { grep -E "FAILED|Error" gpurun_out/ba_tests.log | head -20; tail -30 gpurun_out/ba_tests.log; exit 1; }
tail -1 gpurun_out/ba_tests.log
for lib in librspl_base.so librspl.so librspl_base.so librspl.so; do
  RSPL_LIB=$lib timeout -k 10 120 python -u tools/bench_ba.py --iters 10 --poses 30 --points 10000 --lines 0 2>&1 | tail -1 | sed "s/^/$lib: /" || exit 1
done
RSPL_BA_PROF=1 timeout -k 10 120 python -u tools/bench_ba.py --iters 5 --poses 30 --points 10000 --lines 0 > /dev/null 2> gpurun_out/c5prof.err || exit 1
grep "ba_prof us" gpurun_out/c5prof.err | tail -3
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline --single-precision > gpurun_out/s2_bench_c5.json 2> gpurun_out/c5.err || { tail -5 gpurun_out/c5.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c5', d['value'], d['ms_per_step'], {k: d['stages_ms_per_step'].get(k) for k in ('sg:sinkhorn', 'sg:gnn x18', 'ba:wall')})" gpurun_out/s2_bench_c5.json
