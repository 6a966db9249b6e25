#!/bin/bash
# PMC passes of the bench, one counter set per rocprofv3 run (MI355X_MICROARCH.md's HBM/rocprofv3 section):
#   * MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CU_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_F16, GRBM_GUI_ACTIVE)
#     -> profiles/$ROUND_pmc_mfma_fp16[_WL].json  (tools/pmc_mfma.py)
#   * HBM traffic (FETCH_SIZE, then WRITE_SIZE)  -> profiles/$ROUND_pmc_traffic_fp16[_WL].json (tools/pmc_traffic.py)
# for each workload in $WORKLOADS (default "c3 c4 c5"; C3 files carry no suffix: bench.py reads them for the
# headline, the side workloads' lines read only their own).  Each pass has its own time limit; the chain stops
# at the first failure.
set -o pipefail
R=$PWD
ROUND=${ROUND:-r06}
WORKLOADS=${WORKLOADS:-"c3 c4 c5"}
STEPS=${PMC_STEPS:-10}
mkdir -p gpurun_out
for WL in $WORKLOADS; do
  SUF=""; [ "$WL" != c3 ] && SUF="_$WL"
  B="$R/bench.py --no-cpu-baseline --single-precision --workload $WL --steps $STEPS --warmup 2 --ba-ktime-steps 0"
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE \
      -d $R/gpurun_out/pmc_mfma_$WL -o run --output-format csv -- python3 $B > /dev/null 2> $R/gpurun_out/pmc_mfma_$WL.err \
      || { echo "pmc mfma $WL failed"; tail -5 $R/gpurun_out/pmc_mfma_$WL.err; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_$WL -o run --output-format csv -- python3 $B \
      > /dev/null 2> $R/gpurun_out/pmc_fetch_$WL.err || { echo "pmc fetch $WL failed"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_$WL -o run --output-format csv -- python3 $B \
      > /dev/null 2> $R/gpurun_out/pmc_write_$WL.err || { echo "pmc write $WL failed"; exit 1; }
  cd $R
  python3 tools/pmc_mfma.py $(find gpurun_out/pmc_mfma_$WL -name '*counter_collection.csv' | head -1) \
      > gpurun_out/${ROUND}_pmc_mfma_fp16$SUF.json || exit 1
  python3 tools/pmc_traffic.py $(find gpurun_out/pmc_fetch_$WL -name '*counter_collection.csv' | head -1) \
      $(find gpurun_out/pmc_write_$WL -name '*counter_collection.csv' | head -1) > gpurun_out/${ROUND}_pmc_traffic_fp16$SUF.json || exit 1
  rm -rf gpurun_out/pmc_mfma_$WL gpurun_out/pmc_fetch_$WL gpurun_out/pmc_write_$WL
  echo "pmc $WL done"
done
