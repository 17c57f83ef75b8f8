#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 rocpd database (rocprofv3 --kernel-trace writes
<dir>/<name>_results.db by default): the --stats kernel table (name, calls, total/avg/min/max ns),
written as CSV, plus a per-compaction summary when --per N divides the counts.
usage: kstats_db.py run_results.db [out.csv] [--per N] [--skip-torch]"""
import csv
import sqlite3
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    per = int(sys.argv[sys.argv.index("--per") + 1]) if "--per" in sys.argv else 0
    if per:
        args = [a for a in args if a != str(per)]
    skip = "--skip-torch" in sys.argv
    c = sqlite3.connect(args[0])
    q = ("select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start), min(d.end - d.start), "
         "max(d.end - d.start) from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
         "group by s.kernel_name order by sum(d.end - d.start) desc")
    rows = [r for r in c.execute(q) if not (skip and ("at::native" in r[0] or "rocclr" in r[0]))]
    total = sum(r[2] for r in rows)
    out = [["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"]]
    for r in rows:
        out.append([r[0], r[1], r[2], round(r[3], 1), round(100.0 * r[2] / total, 2), r[4], r[5]])
    if len(args) > 1:
        with open(args[1], "w", newline="") as f:
            csv.writer(f).writerows(out)
    for r in rows:
        line = f"{r[0][:70]:70s} {r[1]:6d} calls {r[3] / 1e3:10.1f} us avg"
        if per:
            line += f" {r[2] / 1e6 / per:9.3f} ms per compaction"
        print(line)


if __name__ == "__main__":
    main()
