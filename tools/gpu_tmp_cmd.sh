#!/bin/bash
# Scratch GPU command of the current experiment (rewritten per experiment).
# Round 5: GNN layer on four workgroups per tile (fixed), warmup with the timed path's instrumentation; the
# driver's command twice, 200-step A/B of the GNN kernels and HEAD's library, the C1 record.
set -o pipefail
mkdir -p gpurun_out/r05b
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_sg.py tests/test_gpu_ba.py -q --timeout 250 --timeout-method thread > gpurun_out/r05b/tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc $rc"; tail -30 gpurun_out/r05b/tests.log; exit 1; fi
grep -E "FAILED|passed|failed" gpurun_out/r05b/tests.log | tail -12
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sg.py -k "c1_fp16 or fp16_vs" -q -s --timeout 250 --timeout-method thread 2>&1 | grep -E "fp16|passed|failed" | head -8
run() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  RSPL_LIB=$lib RSPL_BENCH_TRACE=gpurun_out/r05b/trace_$tag.json timeout -k 10 240 python3 bench.py "$@" \
    > gpurun_out/r05b/$tag.json 2> gpurun_out/r05b/$tag.err || { echo "bench $tag failed"; tail -20 gpurun_out/r05b/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stages_ms_per_step']
print(sys.argv[2], d['value'], d['ms_per_step'], 'ba', s.get('ba:wall'), 'gnn', s.get('sg:gnn x18'), 'sink', s.get('sg:sinkhorn'), 'roof', d['roofline']['kernel'], d['roofline']['frac'])" gpurun_out/r05b/$tag.json $tag
}
run drv1 librspl.so --gpus 1 --steps 20 --warmup 5
run drv2 librspl.so --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
RSPL_SG_GNN=tile1 run drv_t1 librspl.so --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
run s200 librspl.so --steps 200 --warmup 10 --no-cpu-baseline --single-precision
RSPL_SG_GNN=tile1 run s200_t1 librspl.so --steps 200 --warmup 10 --no-cpu-baseline --single-precision
run s200_base librspl_base.so --steps 200 --warmup 10 --no-cpu-baseline --single-precision
RSPL_SG_GNN=tile1 run s200_t1b librspl.so --steps 200 --warmup 10 --no-cpu-baseline --single-precision
run s200b librspl.so --steps 200 --warmup 10 --no-cpu-baseline --single-precision
timeout -k 10 500 python -u tools/run_c1_plumbing.py --pairs 100 --out gpurun_out/r05b/c1_pairs.jsonl > gpurun_out/r05b/c1_plumbing.json 2> gpurun_out/r05b/c1.err || { echo "c1 failed"; tail -5 gpurun_out/r05b/c1.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05b/c1_plumbing.json')); print({k: d[k] for k in d if 'e2e' in k or 'unexpl' in k or 'P_max' in k or 'identical' in k})"
timeout -k 10 120 python -u tools/bench_ba.py --iters 10 --poses 30 --points 10000 --lines 0 > gpurun_out/r05b/c5ba.txt 2>&1 || { echo "c5 ba failed"; tail gpurun_out/r05b/c5ba.txt; exit 1; }
echo "c5 ba: $(tail -1 gpurun_out/r05b/c5ba.txt)"
timeout -k 10 120 python -u tools/bench_ba.py --iters 30 > gpurun_out/r05b/c3ba.txt 2>&1 || { echo "c3 ba failed"; exit 1; }
echo "c3 ba: $(tail -1 gpurun_out/r05b/c3ba.txt)"
