#!/bin/bash
# C5 backward substitution: unconditional operand loads (no exec mask -> exact LDS waits), two steps per iteration
# with ping-pong operands.  Micro-bench variants, BA GPU tests, bitwise A/B of BA results, C5 BA alternating, C5 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 ./tools/experiments/build/solve_bench 29 100 > gpurun_out/sb.txt 2>&1 || { tail -5 gpurun_out/sb.txt; exit 1; }
grep "backward substitution" gpurun_out/sb.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_large.py tests/test_gpu_ba_shard.py tests/test_gpu_map.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 \
    || { grep -E "FAILED|Error" gpurun_out/ba_tests.log | head -20; tail -30 gpurun_out/ba_tests.log; exit 1; }
tail -1 gpurun_out/ba_tests.log
RSPL_LIB=librspl_base.so timeout -k 10 120 python -u tools/experiments/ba_dump.py gpurun_out/ba_base.npz || exit 1
RSPL_LIB=librspl.so timeout -k 10 120 python -u tools/experiments/ba_dump.py gpurun_out/ba_new.npz || exit 1
python3 tools/experiments/frame_pnp_cmp.py gpurun_out/ba_base.npz gpurun_out/ba_new.npz | tail -1
for lib in librspl_base.so librspl.so librspl_base.so librspl.so; do
  RSPL_LIB=$lib timeout -k 10 120 python -u tools/bench_ba.py --iters 10 --poses 30 --points 10000 --lines 0 2>&1 | tail -1 | sed "s/^/$lib: /" || exit 1
done
RSPL_BA_PROF=1 timeout -k 10 120 python -u tools/bench_ba.py --iters 5 --poses 30 --points 10000 --lines 0 > /dev/null 2> gpurun_out/c5prof.err || exit 1
grep "ba_prof us" gpurun_out/c5prof.err | tail -2
for r in 1 2; do
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline --single-precision > gpurun_out/r06_bench_c5_bs$r.json 2> gpurun_out/c5.err || { tail -5 gpurun_out/c5.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c5', d['value'], d['ms_per_step'], d['stages_ms_per_step'].get('ba:wall'))" gpurun_out/r06_bench_c5_bs$r.json
done
