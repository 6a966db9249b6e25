set -o pipefail
for r in 1 2; do for lib in librspl_d4.so librspl_d6.so librspl_d8.so; do
  RSPL_LIB=$lib timeout -k 10 120 python -u tools/bench_ba.py --iters 10 --poses 30 --points 10000 --lines 0 2>&1 | tail -1 | sed "s/^/$lib: /" || exit 1
done; done
for lib in librspl_d4.so librspl_d8.so; do
  RSPL_LIB=$lib timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline --single-precision > gpurun_out/c5_$lib.json 2> gpurun_out/c5.err || { tail -5 gpurun_out/c5.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['stages_ms_per_step'].get('ba:wall'))" gpurun_out/c5_$lib.json
done
