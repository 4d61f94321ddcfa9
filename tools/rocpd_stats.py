"""Kernel statistics (rocprofv3 --kernel-trace --stats) from a rocpd SQLite
database -> CSV (name, calls, total_us, average_us, percent; the view reports microseconds), the summary
committed under profiles/.

    python tools/rocpd_stats.py gpurun_out/prof13/run_results.db profiles/r01_v5_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
        for r in rows:
            w.writerow(r)
    for r in rows[:12]:
        print(f"{r[1]:6d} {r[3]:10.2f} us  {r[4]:5.1f}%  {r[0][:90]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
