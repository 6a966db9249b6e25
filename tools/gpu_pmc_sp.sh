#!/bin/bash
# SQ counters of the SuperPoint kernels (one counter set per rocprofv3 pass).
set -o pipefail
R=$PWD
mkdir -p gpurun_out/pmc_sp
timeout -k 10 120 python tools/bench_sp.py --iters 5 || exit 1
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/pmc_sp/p$i -o run --output-format csv -- python3 $R/tools/bench_sp.py --iters 3 > /dev/null 2>&1 || { echo "pass $i failed"; exit 1; }
done
cd $R
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/pmc_sp/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r['Kernel_Name'][:60]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in acc.items():
    print(k)
    print('   ', {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
