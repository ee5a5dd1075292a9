#!/usr/bin/env python3
"""Kernel summary (name, calls, total/avg duration) from a rocprofv3 rocpd SQLite database, in the
column layout of rocprofv3's kernel_stats.csv:  python tools/rocpd_stats.py run_results.db out.csv"""
import csv
import sqlite3
import sys


def main(db: str, out: str) -> None:
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                          "from kernels group by name order by sum(duration) desc"))
    total = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, n, tot, avg, mn, mx in rows:
            w.writerow([name, n, tot, avg, 100.0 * tot / total, mn, mx])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
