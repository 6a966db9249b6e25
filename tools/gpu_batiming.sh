#!/bin/bash
export RSPL_BA_TIMING=1
timeout -k 10 200 python -u tools/bench_ba.py --iters 20 > gpurun_out/bt_alone.out 2> gpurun_out/bt_alone.err || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision --steps 40 --reserve-cus 0 > gpurun_out/bt_pipe.out 2> gpurun_out/bt_pipe.err || exit 1
python3 - <<'PY'
import re, numpy as np
for f in ("gpurun_out/bt_alone.err", "gpurun_out/bt_pipe.err"):
    rows = [list(map(float, re.findall(r"([a-z0-9]+) ([0-9.]+)", l) and [v for _, v in re.findall(r"([a-z0-9]+) ([0-9.]+)", l)])) for l in open(f) if l.startswith("rspl_ba_local")]
    a = np.array(rows[5:])
    print(f, len(a), "mean us prep csr opt1 classify active2 opt2 final:", a.mean(0).round(0), "total", a.sum(1).mean().round(0))
PY
cat gpurun_out/bt_alone.out; cut -c1-200 gpurun_out/bt_pipe.out
