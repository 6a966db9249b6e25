#!/bin/bash
# BA in-kernel trial spans inside the pipeline under CU reservation / GEMM variants.
export RSPL_BA_PROF=1
run() {  # name, env, bench args
  env $2 timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision --steps 40 $3 > gpurun_out/bc_$1.out 2> gpurun_out/bc_$1.err || exit 1
  python3 - "$1" <<'PY'
import json, re, sys, numpy as np
n = sys.argv[1]
rows = [[float(v) for v in re.findall(r"(-?[0-9.]+)", l.split(":", 1)[1])] for l in open(f"gpurun_out/bc_{n}.err") if l.startswith("ba_prof")]
a = np.median(np.array(rows[5:]), 0).round(1)
d = json.loads(open(f"gpurun_out/bc_{n}.out").read())
s = d["stages_ms_per_step"]
print(f"{n:10s} fps {d['value']:.1f} ba {s['ba:wall']:.3f} gnn {s['sg:gnn x18']:.3f} | pc_st {a[0]} pc {a[1]} asm {a[3]} fac {a[4]} back {a[5]} poses {a[6]} ue_st {a[8]} ue {a[9]}")
PY
}
for cfg in ${CONFIGS:-"base|X=1|"}; do IFS="|" read -r n e a <<< "$cfg"; run "$n" "$e" "$a" || exit 1; done
