#!/bin/bash
# Round evidence, part 1 (ROUND, default r06): GPU tests, smoke, the PMC passes of the headline bench (MFMA busy,
# FETCH_SIZE, WRITE_SIZE: tools/gpu_pmc.sh -> gpurun_out/$ROUND_pmc_{mfma,traffic}_fp16.json, copied to
# profiles/ by hand: bench.py reads them for `traffic` / `mfma_busy`), the headline bench line (200 steps, CPU
# baseline), the driver's shape (20 / 5) three times, and rocprof kernel stats of the bench.  Part 2 (side
# benches) is tools/gpu_round_side.sh.  Everything lands in gpurun_out/ (merged back).  Each GPU step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
R=$PWD
ROUND=${ROUND:-r06}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
fi
if [ -z "$SKIP_PMC" ]; then
ROUND=$ROUND WORKLOADS=${PMC_WORKLOADS:-c3} bash tools/gpu_pmc.sh || exit 1
fi
timeout -k 10 600 python -u bench.py > gpurun_out/${ROUND}_bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/${ROUND}_bench.json
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${ROUND}_bench_driver20_$i.json 2> gpurun_out/bench20.err || { echo "bench 20 failed"; tail -30 gpurun_out/bench20.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('driver-shaped', d['value'], d['ms_per_step'])" gpurun_out/${ROUND}_bench_driver20_$i.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --no-cpu-baseline --single-precision > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || { echo "prof failed"; tail -30 $R/gpurun_out/prof_bench.err; exit 1; }
cd $R
python3 tools/prof_stats.py gpurun_out/prof_bench/run_results.db > gpurun_out/${ROUND}_bench_kernel_stats_fp16.csv
rm -rf gpurun_out/prof_bench
head -12 gpurun_out/${ROUND}_bench_kernel_stats_fp16.csv | cut -c1-150
