#!/bin/bash
# Scratch GPU command of the current experiment (rewritten per experiment).
# Round 5, item 1: the driver's exact bench command (20 steps, warmup 5) with the host timeline
# (RSPL_BENCH_TRACE) on HEAD's library (librspl_base.so) and the working tree's (staging slots, scratch and
# timing events allocated up front), then the 200-step runs for the steady state.
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ba.py -q --timeout 120 --timeout-method thread > gpurun_out/r05/ba_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "BA tests rc $rc"; tail -30 gpurun_out/r05/ba_tests.log; exit 1; fi
grep -E "FAILED|passed|failed" gpurun_out/r05/ba_tests.log | tail -12
tail -1 gpurun_out/r05/ba_tests.log
echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)  nproc: $(nproc)  $(grep Cpus_allowed_list /proc/self/status)"
run() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  RSPL_LIB=$lib RSPL_BENCH_TRACE=gpurun_out/r05/trace_$tag.json timeout -k 10 240 python3 bench.py "$@" \
    > gpurun_out/r05/$tag.json 2> gpurun_out/r05/$tag.err || { echo "bench $tag failed"; tail -20 gpurun_out/r05/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stages_ms_per_step']
print(sys.argv[2], d['value'], d['ms_per_step'], 'ba', s.get('ba:wall'), 'queue', d['host_ms_per_step'].get('ba_queue'))" gpurun_out/r05/$tag.json $tag
}
run new20a librspl.so --gpus 1 --steps 20 --warmup 5
run base20a librspl_base.so --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
run new20b librspl.so --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
run base20b librspl_base.so --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
run new200 librspl.so --steps 200 --warmup 10 --no-cpu-baseline --single-precision
run base200 librspl_base.so --steps 200 --warmup 10 --no-cpu-baseline --single-precision
timeout -k 10 200 python3 -u tools/ba_parity_cases.py > gpurun_out/r05/parity_new.jsonl 2>&1 || { echo "parity failed"; tail gpurun_out/r05/parity_new.jsonl; exit 1; }
timeout -k 10 200 python3 -u tools/ba_parity_cases.py --analytic > gpurun_out/r05/parity_analytic.jsonl 2>&1 || { echo "parity analytic failed"; tail gpurun_out/r05/parity_analytic.jsonl; exit 1; }
echo parity done
timeout -k 10 500 python -u tools/run_c1_plumbing.py --pairs 100 --out gpurun_out/r05/c1_pairs.jsonl > gpurun_out/r05/c1_plumbing.json 2> gpurun_out/r05/c1.err || { echo "c1 failed"; tail -5 gpurun_out/r05/c1.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05/c1_plumbing.json')); print({k: d[k] for k in d if 'e2e' in k or 'unexpl' in k or 'P_max' in k})"
for v in reg packed; do
  [ $v = packed ] && export RSPL_BA_SOLVE_LDS=packed
  timeout -k 10 120 python -u tools/bench_ba.py --iters 10 --poses 30 --points 10000 --lines 0 > gpurun_out/r05/c5ba_$v.txt 2>&1 || { echo "c5 ba $v failed"; tail gpurun_out/r05/c5ba_$v.txt; exit 1; }
  echo "c5 ba $v: $(tail -2 gpurun_out/r05/c5ba_$v.txt)"
done
unset RSPL_BA_SOLVE_LDS
