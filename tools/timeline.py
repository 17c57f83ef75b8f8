"""Timeline of the last bench step from a rocprofv3 kernel trace: each kernel's start offset,
duration and the idle gap before it (host syncs and launch latency show up as gaps).

usage: python tools/timeline.py gpurun_out/prof/run_kernel_trace.csv [first_kernel_substring]
"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2] if len(sys.argv) > 2 else "k_run_header"
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
if not starts:
    sys.exit("no step found")
i0 = starts[-1]
i1 = len(rows)
t0 = int(rows[i0]["Start_Timestamp"])
prev_end = t0
busy = gaps = 0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = max(0, s - prev_end)
    busy += e - s
    gaps += gap
    print(f"{(s - t0) / 1e3:9.1f} us  +gap {gap / 1e3:7.1f}  dur {(e - s) / 1e3:8.1f}  {r['Kernel_Name'][:70]}")
    prev_end = max(prev_end, e)
print(f"span {(prev_end - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, gaps {gaps / 1e3:.1f} us")
