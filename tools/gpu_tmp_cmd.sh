#!/bin/bash
# Scratch GPU command of the current experiment (rewritten per experiment).
# Round 5: point-edge pose blocks recomputed in the diagonal Schur chunks (no per-edge Hpp / bp records),
# reg-solve with unconditional tile loads and a register back-substitution; BA tests, C3 / C5 timings,
# the driver-shaped bench and the PMC traffic of the BA kernels.
set -o pipefail
R=$PWD
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ba.py tests/test_gpu_ba_shard.py tests/test_gpu_map.py tests/test_gpu_pnp.py tests/test_gpu_frame.py -x -v --timeout 250 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
RSPL_BA_PROF=1 timeout -k 10 120 python -u tools/bench_ba.py --iters 4 --poses 30 --points 10000 --lines 0 > $O/c5prof.txt 2>&1 || { echo "c5 prof failed"; tail $O/c5prof.txt; exit 1; }
grep -E "ba_prof|BA " $O/c5prof.txt | tail -3
RSPL_BA_PROF=1 timeout -k 10 120 python -u tools/bench_ba.py --iters 4 > $O/c3prof.txt 2>&1 || { echo "c3 prof failed"; tail $O/c3prof.txt; exit 1; }
grep -E "ba_prof|BA " $O/c3prof.txt | tail -3
RSPL_BA_PROF=1 RSPL_LIB=librspl_base.so timeout -k 10 120 python -u tools/bench_ba.py --iters 4 > $O/c3base.txt 2>&1 || { echo "c3 base failed"; tail $O/c3base.txt; exit 1; }
grep -E "ba_prof|BA " $O/c3base.txt | tail -2
RSPL_LIB=librspl_base.so timeout -k 10 120 python -u tools/bench_ba.py --iters 4 --poses 30 --points 10000 --lines 0 > $O/c5base.txt 2>&1 || { echo "c5 base failed"; tail $O/c5base.txt; exit 1; }
grep -E "BA " $O/c5base.txt | tail -1
RSPL_BENCH_TRACE=$O/trace_drv.json timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --single-precision --no-cpu-baseline > $O/drv.json 2> $O/drv.err || { echo "bench failed"; tail -20 $O/drv.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stages_ms_per_step']
print('drv', d['value'], d['ms_per_step'], 'ba', s.get('ba:wall'))" $O/drv.json
python3 tools/bench_trace.py $O/trace_drv.json | sed -n 3p
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --single-precision --steps 10 --warmup 2 > /dev/null 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_write -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --single-precision --steps 10 --warmup 2 > /dev/null 2>&1 || { echo "pmc write failed"; exit 1; }
cd $R
python3 tools/pmc_traffic.py $(find $O/pmc_fetch -name '*counter_collection.csv' | head -1) $(find $O/pmc_write -name '*counter_collection.csv' | head -1) > $O/pmc_traffic.json || exit 1
rm -rf $O/pmc_fetch $O/pmc_write
python3 -c "
import json; d=json.load(open('$O/pmc_traffic.json'))
for k,v in d.items():
  if 'ba::' in k: print(k[:50], v['launches'], round(v['read_bytes']/1e6,2), round(v['write_bytes']/1e6,2))
"
RSPL_PNP_PROF=1 timeout -k 10 120 python -u tools/bench_frame.py --batch 1 --iters 20 > $O/frame.txt 2>&1 || { echo "frame failed"; tail $O/frame.txt; exit 1; }
grep pnp_prof $O/frame.txt | tail -2; tail -3 $O/frame.txt
