#!/bin/bash
# Where does the local BA lose time in the C3 pipeline?  (1) a rocprofv3 kernel trace of the headline
# bench, analysed by tools/experiments/ba_overlap.py (BA trial kernels alone vs overlapped by each front-end kernel
# class); (2) the bench with stages left out (diagnostics: --skip), BA wall per call in each.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o tl -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --single-precision > gpurun_out/tl_bench.json 2> gpurun_out/tl.err || { echo "trace failed"; tail -5 gpurun_out/tl.err; exit 1; }
python3 tools/experiments/ba_overlap.py gpurun_out/tl > gpurun_out/ba_overlap.txt || exit 1
cat gpurun_out/ba_overlap.txt
for sk in none lines sp,lines sg,lines sp,sg,lines; do
  timeout -k 10 200 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --single-precision --skip $sk > gpurun_out/skip_$sk.json 2> gpurun_out/skip.err || { echo "skip $sk failed"; tail -5 gpurun_out/skip.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['stages_ms_per_step'].get('ba:wall'), d.get('host_ms_per_step'))" gpurun_out/skip_$sk.json $sk
done
bash tools/experiments/gpu_reserve_sweep.sh
