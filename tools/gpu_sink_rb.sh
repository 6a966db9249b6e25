#!/bin/bash
# Row-block Sinkhorn (one exchange per iteration): SG parity tests (expf and the v_exp_f32 variant),
# standalone SG timing + per-phase probe for the slab kernel vs the row-block kernel at several
# workgroups per pair, then a pipeline A/B (frames/s, Sinkhorn, BA wall).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sg.py tests/test_gpu_large.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sink_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/sink_tests.log; exit 1; }
tail -2 gpurun_out/sink_tests.log
for G in 16 32; do
  RSPL_SG_RB_G=$G RSPL_SG_FEXP=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_sg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sink_tests_fx.log 2>&1 && echo "fexp G=$G tests ok" || { echo "fexp G=$G tests FAILED"; grep -E "assert|Error|mismatch" gpurun_out/sink_tests_fx.log | head -8; }
done
for V in ${SINK_VARIANTS:-slab 8 16 32 16fx 32fx}; do
  unset RSPL_SG_SINK RSPL_SG_RB_G RSPL_SG_FEXP
  case $V in slab) export RSPL_SG_SINK=slab;; *fx) export RSPL_SG_RB_G=${V%fx} RSPL_SG_FEXP=1;; *) export RSPL_SG_RB_G=$V;; esac
  echo "== $V"
  timeout -k 10 60 python -u tools/bench_sg.py --precision fp16 --iters 100 || exit 1
  RSPL_SG_PROBE=1 timeout -k 10 60 python -u tools/bench_sg.py --precision fp16 --iters 2 2>&1 | grep cycles | tail -1 || exit 1
done
for rep in 1 2; do
  for V in ${PIPE_VARIANTS:-slab 8 16 16fx}; do
    unset RSPL_SG_SINK RSPL_SG_RB_G RSPL_SG_FEXP
    case $V in slab) export RSPL_SG_SINK=slab;; *fx) export RSPL_SG_RB_G=${V%fx} RSPL_SG_FEXP=1;; *) export RSPL_SG_RB_G=$V;; esac
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision --steps 200 > gpurun_out/sk_ab.json 2> gpurun_out/sk_ab.err || { echo "bench failed"; tail -20 gpurun_out/sk_ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/sk_ab.json')); s=d['stages_ms_per_step']; print(sys.argv[1], d['value'], 'sink', s['sg:sinkhorn'], 'ba', s['ba:wall'], 'roof', d['roofline']['frac'])" $V
  done
done
