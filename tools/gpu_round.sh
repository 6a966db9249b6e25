#!/bin/bash
# Round evidence, part 1 (ROUND, default r03): GPU tests, smoke, the PMC HBM-traffic passes of the
# bench (FETCH_SIZE and WRITE_SIZE in separate runs) -> profiles/$ROUND_pmc_traffic_fp16.json (read by
# bench.py for `traffic`), the headline bench line, and rocprof kernel stats of the bench.  Part 2
# (side benches) is tools/gpu_round_side.sh.  Everything lands in gpurun_out/ (merged back).  Each
# GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=$PWD
ROUND=${ROUND:-r04}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
fi
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --single-precision --steps 10 --warmup 2 > /dev/null 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --single-precision --steps 10 --warmup 2 > /dev/null 2>&1 || { echo "pmc write failed"; exit 1; }
cd $R
python3 tools/pmc_traffic.py $(find gpurun_out/pmc_fetch -name '*counter_collection.csv' | head -1) $(find gpurun_out/pmc_write -name '*counter_collection.csv' | head -1) > gpurun_out/${ROUND}_pmc_traffic_fp16.json || exit 1
cp gpurun_out/${ROUND}_pmc_traffic_fp16.json profiles/${ROUND}_pmc_traffic_fp16.json
timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --no-cpu-baseline --single-precision > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || { echo "prof failed"; tail -30 $R/gpurun_out/prof_bench.err; exit 1; }
cd $R
python3 tools/prof_stats.py gpurun_out/prof_bench/run_results.db > gpurun_out/${ROUND}_bench_kernel_stats_fp16.csv
rm -rf gpurun_out/prof_bench gpurun_out/pmc_fetch gpurun_out/pmc_write
head -12 gpurun_out/${ROUND}_bench_kernel_stats_fp16.csv | cut -c1-150
