#!/bin/bash
# SG fp16 per-kernel stats for each GNN GEMM variant (RSPL_SG_GEMM).
R=$PWD
cd /tmp && export TMPDIR=/tmp
for v in lds rd1 rd2 rk1 rk2; do
  RSPL_SG_GEMM=$v timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_sg_$v -o run -- python3 $R/tools/bench_sg.py --precision fp16 --iters 20 > $R/gpurun_out/sg_$v.log 2>&1 || exit 1
  echo "== $v"; grep ms/call $R/gpurun_out/sg_$v.log | cut -c1-200
  python3 $R/tools/prof_timeline.py $R/gpurun_out/prof_sg_$v/run_results.db | grep -E "gemm_(rd|rk|hh)|attn_h"
done
