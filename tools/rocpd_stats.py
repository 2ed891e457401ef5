#!/usr/bin/env python3
"""Write the per-kernel summary of a rocprofv3 SQLite output (``*_results.db``, the default output
format) as the CSV that ``rocprofv3 --stats --output-format csv`` would give:
Name, Calls, TotalDurationNs, AverageNs, Percentage.

    python tools/rocpd_stats.py gpurun_out/prof/x_results.db profiles/r01_x_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for name, n, tot, avg, pct in rows:  # top_kernels holds microseconds
            w.writerow([name, int(n), float(tot) * 1e3, float(avg) * 1e3, float(pct)])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
