#!/bin/bash
# Stream-priority variants of the bench (the BA stream is always high).
for cfg in "sp=normal,sg=high,post=high" "sp=low,sg=high,post=high" "sp=low,sg=normal,post=normal" "sp=normal,sg=normal,post=normal" "sp=low,sg=low,post=low"; do
  RSPL_STREAM_PRIO=$cfg timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision --steps 60 > gpurun_out/prio.json 2>/dev/null || exit 1
  python3 tools/prio_line.py "$cfg"
done
