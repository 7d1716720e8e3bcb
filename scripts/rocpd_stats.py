"""Per-kernel duration summary from a rocprofv3 rocpd database (the default output of
`rocprofv3 --kernel-trace --stats` on ROCm 7): name, calls, total / average / min / max ns.

    python scripts/rocpd_stats.py gpurun_out/prof/run_results.db [out.csv]
"""
import csv
import sqlite3
import sys



def kernel_rows(db, full=False):
    """[(name, calls, total ns, average ns[, min, max])] by total time, largest first."""
    rows = db.execute(
        "select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start), min(d.end - d.start), max(d.end - d.start) "
        "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
        "group by s.kernel_name order by sum(d.end - d.start) desc").fetchall()
    return rows if full else [r[:4] for r in rows]


if __name__ == "__main__":
    rows = kernel_rows(sqlite3.connect(sys.argv[1]), full=True)
    tot = sum(r[2] for r in rows) or 1
    out = csv.writer(open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout)
    out.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, t, a, lo, hi in rows:
        out.writerow([name, n, t, f"{a:.1f}", f"{100 * t / tot:.2f}", lo, hi])
