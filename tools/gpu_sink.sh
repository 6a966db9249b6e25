#!/bin/bash
timeout -k 10 400 python -u -m pytest tests/test_gpu_sg.py tests/test_gpu_large.py -k "sg or SG or sinkhorn" -x -q --timeout 200 --timeout-method thread > gpurun_out/sg_tests.log 2>&1 || { tail -30 gpurun_out/sg_tests.log; exit 1; }
tail -2 gpurun_out/sg_tests.log
for sk in "" "sg"; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision --steps 40 --skip "$sk" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms_per_step']; print('skip=$sk', d['value'], d['ms_per_step'], s['ba:wall'], s.get('sg:sinkhorn'), s.get('sg:gnn x18'))" || exit 1
done
