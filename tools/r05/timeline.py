"""Per-launch timeline of the last compaction in a rocprofv3 kernel trace (run_kernel_trace.csv):
start offset, gap before, duration, kernel. usage: timeline.py trace.csv [first_kernel_substring]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "skv::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2] if len(sys.argv) > 2 else "k_run_header"
idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
a = idx[-1]
t0 = int(rows[a]["Start_Timestamp"])
prev = None
tot_gap = 0.0
for r in rows[a:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    nm = r["Kernel_Name"].split("(")[0].replace("void ", "")
    gap = (s - prev) / 1e3 if prev else 0.0
    tot_gap += max(gap, 0)
    print(f"{(s - t0) / 1e3:9.1f} +{gap:7.1f} {(e - s) / 1e3:9.1f} us  {nm}")
    prev = e
print(f"span {(prev - t0) / 1e3:.1f} us, gaps {tot_gap:.1f} us")
