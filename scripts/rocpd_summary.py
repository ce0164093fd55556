"""Summarise a rocprofv3 --kernel-trace --stats database (rocpd SQLite) as CSV.

usage: python scripts/rocpd_summary.py <results.db> > profiles/<name>.csv
Columns: kernel, calls, total_us, avg_us, pct (the rocprofv3 `top_kernels` view).
"""
import csv
import sqlite3
import sys


def main(path):
    con = sqlite3.connect(path)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "calls", "total_us", "avg_us", "pct"])
    for name, calls, tot, avg, pct in con.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels"):
        w.writerow([name, calls, round(tot, 3), round(avg, 3), round(pct, 2)])


if __name__ == "__main__":
    main(sys.argv[1])
