#!/bin/bash
# Round-2 close: SG parity first (row-block Sinkhorn; expf default, v_exp_f32 variant checked too), then the round evidence
# (tools/gpu_round.sh), then the Sinkhorn variant sweep for the record.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sink_tests.log 2>&1 || { echo "sg tests FAILED"; grep -E "^E |FAIL" gpurun_out/sink_tests.log | head -12; exit 1; }
tail -1 gpurun_out/sink_tests.log
RSPL_SG_FEXP=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_sg.py tests/test_gpu_large.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sink_tests_fx.log 2>&1 && echo "v_exp_f32 SG tests ok" || { echo "v_exp_f32 SG tests FAILED"; grep -E "^E " gpurun_out/sink_tests_fx.log | head -8; }
bash tools/gpu_round.sh || exit 1
for V in slab 16 16x 13x; do
  unset RSPL_SG_SINK RSPL_SG_RB_G RSPL_SG_FEXP
  case $V in slab) export RSPL_SG_SINK=slab;; *x) export RSPL_SG_RB_G=${V%x} RSPL_SG_FEXP=1;; *) export RSPL_SG_RB_G=$V;; esac
  echo "== $V $(timeout -k 10 60 python -u tools/bench_sg.py --precision fp16 --iters 100 | grep -o "'sinkhorn': [0-9.]*")" || exit 1
done
for rep in 1 2; do
  for V in slab 16 16x; do
    unset RSPL_SG_SINK RSPL_SG_RB_G RSPL_SG_FEXP
    case $V in slab) export RSPL_SG_SINK=slab;; *x) export RSPL_SG_RB_G=${V%x} RSPL_SG_FEXP=1;; *) export RSPL_SG_RB_G=$V;; esac
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision --steps 200 > gpurun_out/sk_ab.json 2> gpurun_out/sk_ab.err || { echo "bench failed"; tail -20 gpurun_out/sk_ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/sk_ab.json')); s=d['stages_ms_per_step']; print(sys.argv[1], d['value'], 'sink', s['sg:sinkhorn'], 'ba', s['ba:wall'], 'roof', d['roofline']['frac'])" $V
  done
done
