RSPL_BA_PROF=1 timeout -k 10 120 python -u tools/bench_ba.py --iters 20 > /dev/null 2> gpurun_out/steps.err || exit 1
grep ba_steps gpurun_out/steps.err | tail -5
