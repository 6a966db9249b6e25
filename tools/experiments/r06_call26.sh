#!/bin/bash
# Schur chunk loop: the next pass's pair index loaded by every lane (clamped) instead of an exec-masked load:
# BA GPU tests, bitwise A/B, standalone C3 BA alternating, in-kernel trace, C3 bench alternating
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_large.py tests/test_gpu_ba_shard.py tests/test_gpu_map.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 \
    || { grep -E "FAILED|Error" gpurun_out/ba_tests.log | head -20; tail -30 gpurun_out/ba_tests.log; exit 1; }
tail -1 gpurun_out/ba_tests.log
RSPL_LIB=librspl_base.so timeout -k 10 120 python -u tools/experiments/ba_dump.py gpurun_out/ba_base.npz || exit 1
RSPL_LIB=librspl.so timeout -k 10 120 python -u tools/experiments/ba_dump.py gpurun_out/ba_new.npz || exit 1
python3 tools/experiments/frame_pnp_cmp.py gpurun_out/ba_base.npz gpurun_out/ba_new.npz | tail -1
for lib in librspl_base.so librspl.so librspl_base.so librspl.so librspl_base.so librspl.so; do
  RSPL_LIB=$lib timeout -k 10 120 python -u tools/bench_ba.py --iters 30 2>&1 | tail -1 | sed "s/^/$lib: /" || exit 1
done
for lib in librspl_base.so librspl.so; do
RSPL_LIB=$lib RSPL_BA_PROF=1 timeout -k 10 120 python -u tools/bench_ba.py --iters 5 > /dev/null 2> gpurun_out/c3prof_$lib.err || exit 1
echo $lib; grep "ba_prof us" gpurun_out/c3prof_$lib.err | tail -1 | cut -c1-120
done
for lib in librspl_base.so librspl.so librspl_base.so librspl.so; do
  RSPL_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab26_$lib.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['stages_ms_per_step'].get('ba:wall'))" gpurun_out/ab26_$lib.json $lib
done
