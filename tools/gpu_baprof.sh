#!/bin/bash
# In-kernel spans of one traced BA trial per call (RSPL_BA_PROF), alone and inside the pipeline.
export RSPL_BA_PROF=1
timeout -k 10 200 python -u tools/bench_ba.py --iters 20 > gpurun_out/bp_alone.out 2> gpurun_out/bp_alone.err || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision --steps 40 > gpurun_out/bp_pipe.out 2> gpurun_out/bp_pipe.err || exit 1
python3 - <<'PY'
import re, numpy as np
for f in ("gpurun_out/bp_alone.err", "gpurun_out/bp_pipe.err"):
    lines = [l for l in open(f) if l.startswith("ba_prof ")]
    names = re.findall(r"([a-z]+) -?[0-9.]+", lines[0].split(":", 1)[1])
    rows = [[float(v) for v in re.findall(r"(-?[0-9.]+)", l.split(":", 1)[1])] for l in lines]
    a = np.median(np.array(rows[5:]), 0).round(1)
    print(f, len(rows), "median us:", " ".join(f"{n}={v}" for n, v in zip(names, a)))
PY
cat gpurun_out/bp_alone.out
