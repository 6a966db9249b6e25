#!/bin/bash
# Round-6 GPU call 1: PMC passes (MFMA busy + traffic, C3/C4/C5), then the 100-keyframe sequence with the
# analytic line Jacobian on both sides and its lockstep divergence check.
set -o pipefail
mkdir -p gpurun_out
ROUND=r06 bash tools/gpu_pmc.sh || exit 1
timeout -k 10 400 python -u tools/run_sequence.py --analytic-line-jacobian --out gpurun_out/seq_analytic \
    > gpurun_out/r06_sequence100_analytic.json 2> gpurun_out/seq_analytic.err || { tail -5 gpurun_out/seq_analytic.err; exit 1; }
cat gpurun_out/r06_sequence100_analytic.json
timeout -k 10 400 python -u tools/sequence_divergence.py --analytic-line-jacobian --show 4 > gpurun_out/seq_div_analytic.log 2>&1 \
    || { tail -5 gpurun_out/seq_div_analytic.log; exit 1; }
cat gpurun_out/seq_div_analytic.log
