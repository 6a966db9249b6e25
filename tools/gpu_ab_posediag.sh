set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_ba_shard.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pd_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pd_tests.log; exit 1; }
tail -1 gpurun_out/pd_tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in librspl_old.so librspl.so; do
  RSPL_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pd_$L -o run -- python3 tools/bench_ba.py --iters 50 > /dev/null 2>&1 || { echo "prof failed"; exit 1; }
  python3 - "$L" <<'PY'
import sqlite3,sys,glob
f=glob.glob(f"gpurun_out/pd_{sys.argv[1]}/**/run_results.db", recursive=True)[0]
c=sqlite3.connect(f)
for n,cnt,avg in c.execute("select name,count(*),avg(duration) from kernels where name like '%pair_chunk%' or name like '%schur%' group by name"):
    print(sys.argv[1], n[:40], cnt, round(avg/1000,2))
PY
  rm -rf gpurun_out/pd_$L
done
bash tools/gpu_lib_ab.sh
