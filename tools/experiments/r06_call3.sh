#!/bin/bash
# Round-6 GPU call 3: per-kernel times of SuperPoint fp16 vs split fp16 (rocprofv3 stats), then the C1 record.
set -o pipefail
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for p in fp16 fp16x3; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sp_$p -o run -- python3 $R/tools/bench_sp.py --precision $p --iters 50 \
      > $R/gpurun_out/prof_sp_$p.txt 2>&1 || { tail -5 $R/gpurun_out/prof_sp_$p.txt; exit 1; }
done
cd $R
for p in fp16 fp16x3; do
  python3 tools/prof_stats.py gpurun_out/prof_sp_$p/run_results.db > gpurun_out/r06_sp_kernel_stats_$p.csv || exit 1
  head -14 gpurun_out/r06_sp_kernel_stats_$p.csv | cut -c1-160
done
rm -rf gpurun_out/prof_sp_fp16 gpurun_out/prof_sp_fp16x3
timeout -k 10 900 python -u tools/run_c1_plumbing.py --out gpurun_out/r06_c1_pairs.jsonl > gpurun_out/r06_c1_plumbing.json 2> gpurun_out/c1.err \
    || { tail -20 gpurun_out/c1.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r06_c1_plumbing.json'));print(d['fp16x3']); print(d['keypoint_overlap_fp16_min'], d['match_agreement_fp16_mean'])"
