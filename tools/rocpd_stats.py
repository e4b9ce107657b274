"""Kernel statistics CSV (the columns of rocprofv3's kernel_stats.csv) from a rocprofv3 rocpd
database, for runs made without --output-format csv (not product).
usage: python tools/rocpd_stats.py run_results.db out.csv"""
import csv
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    with open(sys.argv[2], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, n, s, a, lo, hi in rows:
            w.writerow([name, n, s, round(a, 1), round(100.0 * s / tot, 4), lo, hi])


if __name__ == "__main__":
    main()
