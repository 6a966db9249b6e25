#!/bin/bash
# bench.py modes on one GPU: the default C3 line, the RCCL-sharded BA mode at N=1, a short C5 run,
# and --gpus 2 on a one-GPU box (must fail loudly, not hang); plus the 2-process sharded-BA test.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ba_shard.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/shard_tests.log 2>&1 || { echo "shard tests failed"; tail -30 gpurun_out/shard_tests.log; exit 1; }
tail -2 gpurun_out/shard_tests.log
timeout -k 10 200 python -u bench.py --ba-mode shard --no-cpu-baseline --single-precision --steps 50 > gpurun_out/bench_shard.json 2> gpurun_out/bench_shard.err || { echo "bench shard failed"; tail -30 gpurun_out/bench_shard.err; exit 1; }
cat gpurun_out/bench_shard.json
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --single-precision --steps 20 --warmup 3 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { echo "bench c5 failed"; tail -30 gpurun_out/bench_c5.err; exit 1; }
cat gpurun_out/bench_c5.json
timeout -k 10 120 python -u bench.py --gpus 2 --no-cpu-baseline --single-precision --steps 5 > gpurun_out/bench_g2.json 2> gpurun_out/bench_g2.err; echo "gpus=2 on one GPU exit code: $?"; tail -3 gpurun_out/bench_g2.err
