#!/bin/bash
# Sinkhorn polling variant: parity, standalone per-G timing + probe, then the pipeline at G=16 / 32.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sg.py tests/test_gpu_large.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sink_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/sink_tests.log; exit 1; }
tail -1 gpurun_out/sink_tests.log
for G in 16 32; do
  RSPL_SG_SINK_G=$G timeout -k 10 60 python -u tools/bench_sg.py --precision fp16 --iters 100 || exit 1
  RSPL_SG_SINK_G=$G RSPL_SG_PROBE=1 timeout -k 10 60 python -u tools/bench_sg.py --precision fp16 --iters 2 2>&1 | tail -1 || exit 1
done
run() {
  env "$@" timeout -k 10 120 python -u bench.py --single-precision --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench failed"; tail -20 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); s=d['stages_ms_per_step']; print(sys.argv[1:], d['value'], 'ba', s['ba:wall'], 'gnn', s['sg:gnn x18'], 'sink', s['sg:sinkhorn'])" "$@"
}
run RSPL_SG_SINK_G=16
run RSPL_SG_SINK_G=32
run RSPL_SG_SINK_G=16
run RSPL_SG_SINK_G=32
