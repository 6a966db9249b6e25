#!/bin/bash
# Round evidence, part 2 (ROUND, default r03): standalone BA (C3, C5), line front end, FrameOptimization /
# PnP, the BASELINE C1 plumbing run (100 stereo pairs, SP/SG/lines vs the CPU restatement) and the
# 100-keyframe map-side sequence -> gpurun_out/${ROUND}_*.  Each step has its own time limit.
set -o pipefail
ROUND=${ROUND:-r06}
mkdir -p gpurun_out
{ timeout -k 10 120 python -u tools/bench_ba.py --iters 50 && timeout -k 10 120 python -u tools/bench_ba.py --iters 10 --poses 30 --points 10000 --lines 0; } > gpurun_out/${ROUND}_bench_ba.txt || { echo "ba bench failed"; exit 1; }
cat gpurun_out/${ROUND}_bench_ba.txt
timeout -k 10 200 python -u tools/bench_lines.py > gpurun_out/${ROUND}_bench_lines.json || { echo "line bench failed"; exit 1; }
cat gpurun_out/${ROUND}_bench_lines.json
timeout -k 10 200 python -u tools/bench_frame.py > gpurun_out/${ROUND}_bench_frame.json 2> gpurun_out/bench_frame.err || { echo "frame bench failed"; tail -5 gpurun_out/bench_frame.err; exit 1; }
cat gpurun_out/${ROUND}_bench_frame.json
timeout -k 10 400 python -u tools/run_c1_plumbing.py --pairs 100 --out gpurun_out/${ROUND}_c1_pairs.jsonl > gpurun_out/${ROUND}_c1_plumbing.json 2> gpurun_out/c1.err || { echo "c1 failed"; tail -5 gpurun_out/c1.err; exit 1; }
cat gpurun_out/${ROUND}_c1_plumbing.json
timeout -k 10 500 python -u tools/run_sequence.py --out gpurun_out/${ROUND}_sequence > gpurun_out/${ROUND}_sequence100.json 2> gpurun_out/seq.err || { echo "sequence failed"; tail -5 gpurun_out/seq.err; exit 1; }
cat gpurun_out/${ROUND}_sequence100.json
timeout -k 10 500 python -u tools/run_sequence.py --analytic-line-jacobian --out gpurun_out/${ROUND}_sequence_analytic > gpurun_out/${ROUND}_sequence100_analytic.json 2> gpurun_out/seqa.err || { echo "sequence (analytic) failed"; tail -5 gpurun_out/seqa.err; exit 1; }
cat gpurun_out/${ROUND}_sequence100_analytic.json
timeout -k 10 300 python -u bench.py --workload c4 --steps 100 --warmup 5 --no-cpu-baseline --single-precision > gpurun_out/${ROUND}_bench_c4.json 2> gpurun_out/c4.err || { echo "c4 bench failed"; tail -5 gpurun_out/c4.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c4', d['value'], d['ms_per_step'])" gpurun_out/${ROUND}_bench_c4.json
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline --single-precision > gpurun_out/${ROUND}_bench_c5.json 2> gpurun_out/c5.err || { echo "c5 bench failed"; tail -5 gpurun_out/c5.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c5', d['value'], d['ms_per_step'], {k: d['stages_ms_per_step'].get(k) for k in ('sg:sinkhorn', 'sg:gnn x18', 'ba:wall')})" gpurun_out/${ROUND}_bench_c5.json
