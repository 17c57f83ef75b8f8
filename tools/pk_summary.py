#!/usr/bin/env python3
"""Per-dispatch durations (last compaction of the trace) and per-kernel PMC sums of a
tools/pmc_counters.sh output directory.  usage: pk_summary.py gpurun_out/pk_<C> [kernel-substr ...]"""
import collections
import csv
import glob
import re
import sys


def short(n):
    n = re.sub(r"^void ", "", n)
    d, o = 0, []
    for ch in n:
        if ch == "(":
            d += 1
        if d == 0:
            o.append(ch)
        if ch == ")":
            d -= 1
    return "".join(o).replace("skv::", "")


def main():
    root = sys.argv[1]
    want = sys.argv[2:]
    rows = [r for r in csv.DictReader(open(f"{root}/trace/run_kernel_trace.csv")) if "skv::" in r["Kernel_Name"]]
    tot = collections.defaultdict(float)
    for r in rows:
        tot[short(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print("kernel total_us (all dispatches in the trace)")
    for k, v in sorted(tot.items(), key=lambda x: -x[1])[:25]:
        print(f"  {k:28s} {v:10.1f}")
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in sorted(glob.glob(f"{root}/g*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if want and not any(w in k for w in want):
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in agg.items():
        print(k, {a: f"{b:.3g}" for a, b in v.items()})


if __name__ == "__main__":
    main()
