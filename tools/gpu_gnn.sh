#!/bin/bash
# Fused GNN layers: SG parity tests (fp16 bar, fp32 untouched), then SG timing fused vs unfused.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sg.py tests/test_gpu_large.py tests/test_abi_c.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gnn_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gnn_tests.log; exit 1; }
tail -1 gpurun_out/gnn_tests.log
for M in unfused fused; do
  RSPL_SG_GNN=$M timeout -k 10 60 python -u tools/bench_sg.py --precision fp16 --iters 100 || exit 1
done
