"""Write a kernel_stats-style CSV (name, calls, total/avg/min/max ns, %) from a rocprofv3
rocpd SQLite database (used when a run produced run_results.db instead of CSVs).

usage: python tools/rocpd_stats.py RESULTS.db OUT.csv
"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), "
                     "max(duration) from kernels group by name order by sum(duration) desc"
                     ).fetchall()
    tot = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
        for n, k, s, a, mn, mx in rows:
            w.writerow([n[:160], k, s, round(a, 1), mn, mx, round(100.0 * s / tot, 2)])


if __name__ == "__main__":
    main()
