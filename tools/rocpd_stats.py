"""Per-kernel stats (rocprofv3 --stats CSV layout: Name,Calls,TotalDurationNs,AverageNs,Percentage)
from a rocprofv3 rocpd SQLite database (the default output of this ROCm build when no
--output-format is given).

    python tools/rocpd_stats.py gpurun_out/.../run_results.db > profiles/rXX_..._kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main():
    con = sqlite3.connect(sys.argv[1])
    rows = con.execute("select name, count(*), sum(end - start), avg(end - start) from kernels "
                       "group by name order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for name, calls, total, avg in rows:
        w.writerow([name, calls, int(total), f"{avg:.3f}", f"{100.0 * total / tot:.4f}"])


if __name__ == "__main__":
    main()
