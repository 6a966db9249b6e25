#!/bin/bash
# BA in-kernel trial spans inside the pipeline for bench variants.
# CONFIGS="name|ENV=val|--arg_--arg2 ..." (underscores in the args become spaces).
export RSPL_BA_PROF=1
run() {  # name, env, bench args
  env $2 timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision --steps 40 ${3//_/ } > gpurun_out/bc_$1.out 2> gpurun_out/bc_$1.err || exit 1
  python3 - "$1" <<'PY'
import json, re, sys, numpy as np
n = sys.argv[1]
lines = [l for l in open(f"gpurun_out/bc_{n}.err") if l.startswith("ba_prof ")]
names = re.findall(r"([a-z]+) -?[0-9.]+", lines[0].split(":", 1)[1])
rows = [[float(v) for v in re.findall(r"(-?[0-9.]+)", l.split(":", 1)[1])] for l in lines]
a = dict(zip(names, np.median(np.array(rows[5:]), 0).round(1)))
d = json.loads(open(f"gpurun_out/bc_{n}.out").read())
s = d["stages_ms_per_step"]
print(f"{n:8s} fps {d['value']:.1f} ba {s['ba:wall']:.3f} gnn {s['sg:gnn x18']:.3f} |", " ".join(f"{k}={a[k]}" for k in ("pcstarts", "pcend", "factor", "poses", "uestarts", "groupsend", "linesend")))
PY
}
for cfg in ${CONFIGS:-"base|X=1|"}; do IFS="|" read -r n e a <<< "$cfg"; run "$n" "$e" "$a" || exit 1; done
