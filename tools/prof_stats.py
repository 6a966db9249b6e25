"""Per-kernel stats from a rocprofv3 rocpd database (`rocprofv3 --kernel-trace --stats -d DIR
-o run` writes DIR/run_results.db), as CSV on stdout: the same columns as rocprofv3's
kernel_stats.csv (durations in ns).
Usage: python tools/prof_stats.py gpurun_out/prof_bench/run_results.db > profiles/rNN_..._kernel_stats.csv"""
import csv
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, calls, tot, avg, mn, mx in rows:
        w.writerow([name, calls, tot, round(avg, 1), round(100.0 * tot / total, 3), mn, mx])


if __name__ == "__main__":
    main()
