"""Kernel statistics (name, calls, total / average / min / max duration in ns, percentage) from a rocprofv3
rocpd database (rocprofv3 --kernel-trace --stats -d DIR -o NAME writes DIR/.../NAME_results.db), written as
CSV like rocprofv3's kernel_stats.csv.  usage: python tools/rocpd_stats.py run_results.db out.csv"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                          "from kernels group by name order by sum(duration) desc"))
    tot = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
        for r in rows:
            w.writerow([r[0], r[1], r[2], round(r[3], 1), r[4], r[5], round(100.0 * r[2] / tot, 4)])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
