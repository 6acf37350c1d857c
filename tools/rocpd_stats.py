#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 rocpd database (the default output of
`rocprofv3 --kernel-trace --stats -d DIR -o run`): name, calls, total/average/min/max ns and
share of summed kernel time, as CSV on stdout (the form committed under profiles/).
Usage: python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/rNN_rocprof_stats.csv"""
import csv
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute(
        "select name, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
        "from kernels group by name order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, tot, avg, mn, mx in rows:
        w.writerow([name, n, int(tot), round(avg, 1), round(100.0 * tot / total, 3), int(mn), int(mx)])


if __name__ == "__main__":
    main(sys.argv[1])
