"""Export the per-kernel summary (`top_kernels` view) of a rocprofv3 rocpd database as the
same columns as rocprofv3's `--stats` kernel_stats.csv (Name, Calls, TotalDurationNs,
AverageNs, Percentage).  ROCm 7.2's rocprofv3 writes the rocpd SQLite format by default.

usage: python tools/rocpd_stats.py gpurun_out/prof/run_results.db profiles/x.csv
"""
import csv
import sqlite3
import sys


def main(db, out):
    con = sqlite3.connect(db)
    rows = con.execute("select name, total_calls, total_duration, average, percentage "
                       "from top_kernels order by total_duration desc").fetchall()
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
        for name, calls, tot, avg, pct in rows:
            w.writerow([name, calls, f"{tot:.3f}", f"{avg:.3f}", f"{pct:.2f}"])
    print(f"{len(rows)} kernels -> {out}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
