"""Kernel statistics (rocprofv3 --stats layout) from a rocprofv3 SQLite database.

    python tools/prof_stats.py gpurun_out/prof/prof_results.db [out.csv]
"""
import csv
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = db.execute("SELECT name, COUNT(*), SUM(end - start), AVG(end - start), MIN(end - start), "
                      "MAX(end - start) FROM kernels GROUP BY name ORDER BY SUM(end - start) DESC"
                      ).fetchall()
    total = sum(r[2] for r in rows) or 1
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, tot, avg, mn, mx in rows:
        w.writerow([name, n, tot, round(avg, 1), round(100.0 * tot / total, 2), mn, mx])


if __name__ == "__main__":
    main()
