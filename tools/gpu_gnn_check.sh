#!/bin/bash
# SuperGlue fused-layer changes: SG parity tests (fp32 exact path, fp16 bar), per-phase layer probe,
# then the pipeline bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sg.py tests/test_gpu_large.py -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/sg_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/sg_tests.log; exit 1; }
grep -E "agree|passed|failed" gpurun_out/sg_tests.log | tail -5
RSPL_SG_LPROBE=1 timeout -k 10 120 python -u tools/bench_sg.py --iters 20 2>&1 | tail -2 || exit 1
timeout -k 10 300 python -u bench.py --single-precision --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['ms_per_step'], d['stages_ms_per_step'])"
RSPL_SG_NOXCD=1 RSPL_SG_LPROBE=1 timeout -k 10 120 python -u tools/bench_sg.py --iters 20 2>&1 | tail -2 | sed 's/^/noxcd: /' || exit 1
RSPL_SG_NOXCD=1 timeout -k 10 300 python -u bench.py --single-precision --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print('noxcd', d['value'], d['ms_per_step'], d['stages_ms_per_step']['sg:gnn x18'], d['stages_ms_per_step']['ba:wall'])"
