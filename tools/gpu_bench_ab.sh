#!/bin/bash
# A/B of bench.py knobs in the pipeline: Sinkhorn workgroups per pair and host- vs device-decided LM.
set -o pipefail
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 120 python -u bench.py --single-precision --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench failed"; tail -20 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); s=d['stages_ms_per_step']; print(sys.argv[1:], d['value'], 'ba', s['ba:wall'], 'gnn', s['sg:gnn x18'], 'sink', s['sg:sinkhorn'])" "$@"
}
run RSPL_SG_SINK_G=16 RSPL_BA_HOSTLM=1
run RSPL_SG_SINK_G=32 RSPL_BA_HOSTLM=1
run RSPL_SG_SINK_G=16 X=1
run RSPL_SG_SINK_G=32 X=1
run RSPL_SG_SINK_G=16 X=2
run RSPL_SG_SINK_G=32 X=2
