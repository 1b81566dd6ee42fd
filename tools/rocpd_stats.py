#!/usr/bin/env python3
"""Per-kernel summary (calls, total/avg/min/max ns, share) from a rocprofv3
rocpd SQLite database -- the same table `rocprofv3 --stats` writes as CSV.

  python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/rNN/kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                          "from kernels group by name order by 3 desc"))
    tot = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, s, a, lo, hi in rows:
        w.writerow([name, n, s, round(a, 1), round(100.0 * s / tot, 2), lo, hi])


if __name__ == "__main__":
    main(sys.argv[1])
