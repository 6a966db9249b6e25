#!/bin/bash
# Scratch GPU command of the current experiment (rewritten per experiment).
# Round 5: the first timed BA call's 7-8 ms stall inside hipMemcpyAsync -- the upload as a kernel vs the
# copy, and a HIP API log of the copy case; the C5 BA solve's phases (in-kernel trace).
set -o pipefail
mkdir -p gpurun_out/r05c
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ba.py tests/test_gpu_sg.py -q -x --timeout 250 --timeout-method thread > gpurun_out/r05c/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r05c/tests.log; exit 1; }
tail -1 gpurun_out/r05c/tests.log
run() {  # tag args...
  local tag=$1; shift
  RSPL_BENCH_TRACE=gpurun_out/r05c/trace_$tag.json timeout -k 10 240 python3 bench.py "$@" \
    > gpurun_out/r05c/$tag.json 2> gpurun_out/r05c/$tag.err || { echo "bench $tag failed"; tail -20 gpurun_out/r05c/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stages_ms_per_step']
print(sys.argv[2], d['value'], d['ms_per_step'], 'ba', s.get('ba:wall'), 'gnn', s.get('sg:gnn x18'))" gpurun_out/r05c/$tag.json $tag
  python3 tools/bench_trace.py gpurun_out/r05c/trace_$tag.json | sed -n 3p
}
run copy --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --single-precision
RSPL_BA_UPLOAD=kernel run kern --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --single-precision
AMD_LOG_LEVEL=4 AMD_LOG_MASK=0x105 run copylog --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --single-precision
grep -c . gpurun_out/r05c/copylog.err
RSPL_BA_UPLOAD=kernel run kern2 --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --single-precision
RSPL_BA_PROF=1 timeout -k 10 120 python -u tools/bench_ba.py --iters 4 --poses 30 --points 10000 --lines 0 > gpurun_out/r05c/c5prof.txt 2>&1 || { echo "c5 prof failed"; tail gpurun_out/r05c/c5prof.txt; exit 1; }
grep -E "ba_prof|BA " gpurun_out/r05c/c5prof.txt | tail -4
