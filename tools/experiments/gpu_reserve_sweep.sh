#!/bin/bash
# C3 bench with the front-end streams (SP / SG / post) CU-masked off R CUs that only the BA stream may
# use besides the rest (--ba-own-cus 0: the BA stream itself unmasked), alternating with the default.
set -o pipefail
mkdir -p gpurun_out
for cfg in "0 0" "16 0" "32 0" "64 0" "0 0" "16 0" "32 0" "64 0"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --steps 150 --warmup 10 --no-cpu-baseline --reserve-cus $1 --ba-own-cus $2 > gpurun_out/rs.json 2> gpurun_out/rs.err || { echo "reserve $1 failed"; tail -5 gpurun_out/rs.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('reserve', sys.argv[2], 'own', sys.argv[3], d['value'], d['ms_per_step'], 'ba', d['stages_ms_per_step'].get('ba:wall'), 'gnn', d['stages_ms_per_step'].get('sg:gnn x18'), 'conv1', d['stages_ms_per_step'].get('sp:conv1a+1b+pool'))" gpurun_out/rs.json $1 $2
done
