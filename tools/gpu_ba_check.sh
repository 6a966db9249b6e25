set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_ba_shard.py tests/test_gpu_large.py tests/test_gpu_map.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ba_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ba_tests.log; exit 1; }
tail -1 gpurun_out/ba_tests.log
timeout -k 10 200 python -u tools/ba_repeat.py > gpurun_out/ba_repeat.log 2>&1 || { echo "repeat failed"; tail -20 gpurun_out/ba_repeat.log; exit 1; }
tail -3 gpurun_out/ba_repeat.log
bash tools/gpu_baprof.sh
timeout -k 10 300 python -u bench.py --single-precision --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['ms_per_step'], d['ba'])"
