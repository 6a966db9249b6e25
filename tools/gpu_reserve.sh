#!/bin/bash
for cfg in "0 0" "16 1" "32 1" "48 1" "32 0"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision --steps 40 --reserve-cus $1 --ba-own-cus $2 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 $2', d['value'], d['ms_per_step'], d['stages_ms_per_step']['ba:wall'], d['stages_ms_per_step']['sg:gnn x18'], d['stages_ms_per_step']['sg:sinkhorn'])" || exit 1
done
