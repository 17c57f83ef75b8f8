"""Summarise rocprofv3 --pmc CSVs per kernel (last dispatch of each kernel = timed step)."""
import csv, glob, sys, collections
root = sys.argv[1]
per = collections.defaultdict(dict)   # kernel -> counter -> list of values
dur = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/g*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        per[k].setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, cs in sorted(per.items(), key=lambda kv: -max(dur[kv[0]])):
    s = ", ".join(f"{c}={v[-1]:.4g}" for c, v in cs.items())
    print(f"{k[:40]:40s} n={len(next(iter(cs.values())))} dur_us(last)={dur[k][-1]:9.1f}  {s}")
