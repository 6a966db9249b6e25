#!/bin/bash
# Row-block Sinkhorn: parity with the v_exp_f32 variant, poll-spacing sweep (standalone), then a
# pipeline A/B of slab / row-block expf / row-block v_exp_f32 (frames/s, Sinkhorn, BA wall).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sg.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sink_tests.log 2>&1 && echo "sg tests ok" || { echo "sg tests FAILED"; grep -E "^E |FAIL" gpurun_out/sink_tests.log | head -12; exit 1; }
RSPL_SG_FEXP=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_sg.py tests/test_gpu_large.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sink_tests_fx.log 2>&1 && echo "fexp tests ok" || { echo "fexp tests FAILED"; grep -E "^E " gpurun_out/sink_tests_fx.log | head -12; }
for G in 13 16; do
  for SL in 1 8; do
    for FX in 0 1; do
      echo "G $G sleep $SL fexp $FX"
      RSPL_SG_RB_G=$G RSPL_SG_SLEEP=$SL RSPL_SG_FEXP=$FX timeout -k 10 60 python -u tools/bench_sg.py --precision fp16 --iters 100 | grep -o "'sinkhorn': [0-9.]*" || exit 1
    done
  done
done
for rep in 1 2 3; do
  for V in ${PIPE_VARIANTS:-slab 16 16fx 13fx}; do
    unset RSPL_SG_SINK RSPL_SG_RB_G RSPL_SG_FEXP
    case $V in slab) export RSPL_SG_SINK=slab;; *fx) export RSPL_SG_RB_G=${V%fx} RSPL_SG_FEXP=1;; *) export RSPL_SG_RB_G=$V;; esac
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision --steps 200 > gpurun_out/sk_ab.json 2> gpurun_out/sk_ab.err || { echo "bench failed"; tail -20 gpurun_out/sk_ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/sk_ab.json')); s=d['stages_ms_per_step']; print(sys.argv[1], d['value'], 'sink', s['sg:sinkhorn'], 'ba', s['ba:wall'], 'roof', d['roofline']['frac'])" $V
  done
done
