"""Kernel summary (the rocprofv3 --kernel-trace --stats table) from a rocprofv3
rocpd SQLite database, written as CSV for profiles/.

Usage: python tools/rocpd_stats.py RUN_RESULTS.db OUT.csv
Columns: Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs,
VGPRs, AGPRs, LDS bytes, grid size (first dispatch).
"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1:3]
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
        "max(vgpr_count), max(accum_vgpr_count), max(lds_size), max(grid_x) from kernels group by name "
        "order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "VGPRs", "AGPRs",
                    "LDSBytes", "GridX"])
        for name, n, tot, avg, mn, mx, vg, ag, lds, gx in rows:
            w.writerow([name, n, tot, round(avg, 1), round(100.0 * tot / total, 2), mn, mx, vg, ag, lds, gx])
    for r in rows[:8]:
        print(f"{100.0 * r[2] / total:6.2f}%  {r[1]:5d} x {r[3] / 1e3:9.1f} us  {r[0].split('(')[0]}")


if __name__ == "__main__":
    main()
