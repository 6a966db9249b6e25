#!/bin/bash
for sk in "" "sg" "sp" "sp,sg"; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision --steps 40 --skip "$sk" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('skip=$sk', d['value'], d['ms_per_step'], d['stages_ms_per_step']['ba:wall'])" || exit 1
done
