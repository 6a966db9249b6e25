set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sg.py -k "c1" -x -v -s --timeout 120 --timeout-method thread > gpurun_out/sg_c1_tests.log 2>&1; tail -15 gpurun_out/sg_c1_tests.log
LIBS="librspl_r03.so librspl.so" BENCH_AB=2 bash tools/gpu_ba_ab.sh || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --single-precision > gpurun_out/b_new.json 2> gpurun_out/b_new.err || { tail -20 gpurun_out/b_new.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/b_new.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d['roofline']))
for k,v in d['stages_roofline'].items(): print(k, v.get('ms'), v['avg_launch_ms'], v['frac'])"
