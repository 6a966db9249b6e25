#!/bin/bash
# Pipeline A/B of the fused GNN layers (RSPL_SG_GNN=unfused vs default), two runs each.
set -o pipefail
mkdir -p gpurun_out
run() {
  env "$@" timeout -k 10 120 python -u bench.py --single-precision --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench failed"; tail -20 gpurun_out/ab.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); s=d['stages_ms_per_step']; print(sys.argv[1:], d['value'], 'ba', s['ba:wall'], 'gnn', s['sg:gnn x18'], 'sink', s['sg:sinkhorn'], 'sp1', s['sp:conv1a+1b+pool'])" "$@"
}
run RSPL_SG_GNN=unfused
run RSPL_SG_GNN=fused
run RSPL_SG_GNN=unfused
run RSPL_SG_GNN=fused
