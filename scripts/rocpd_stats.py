"""Per-kernel stats CSV (rocprofv3 --stats layout) from a rocprofv3 SQLite results database.

Usage: python scripts/rocpd_stats.py <run_results.db> <out.csv>
"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute("""select s.display_name, count(*), sum(d.end - d.start), avg(d.end - d.start),
                               min(d.end - d.start), max(d.end - d.start)
                        from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
                        group by s.display_name order by sum(d.end - d.start) desc""").fetchall()
    tot = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for r in rows:
            w.writerow([r[0], r[1], r[2], round(r[3], 1), round(100 * r[2] / tot, 4), r[4], r[5]])
    return rows


if __name__ == "__main__":
    for r in main(sys.argv[1], sys.argv[2]):
        if "build_operand" in r[0] or "spmm_unit_kernel<4, 16" in r[0]:
            print(r[1], round(r[3] / 1e3, 1), r[4] / 1e3, r[5] / 1e3, r[0][:90])
