#!/bin/bash
# L2 hit / miss and HBM fetch of the GNN layer kernels (both schedules), SuperGlue alone
set -o pipefail
R=$PWD
mkdir -p gpurun_out/pmc_gnn
timeout -k 10 120 python tools/bench_sg.py --iters 3 > /dev/null || exit 1
cd /tmp && export TMPDIR=/tmp
for m in quad fused8; do
  i=0
  for set in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
    i=$((i+1))
    RSPL_SG_GNN=$m timeout -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/pmc_gnn/${m}_p$i -o run --output-format csv -- python3 $R/tools/bench_sg.py --iters 3 > /dev/null 2>&1 || { echo "pass $m $i failed"; exit 1; }
  done
done
cd $R
python3 - <<'PY'
import csv, glob, collections
for m in ("quad", "fused8"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f'gpurun_out/pmc_gnn/{m}_p*/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'layer' in r['Kernel_Name']:
                acc[r['Kernel_Name'][:40]][r['Counter_Name']].append(float(r['Counter_Value']))
    for k, d in acc.items():
        print(m, k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
