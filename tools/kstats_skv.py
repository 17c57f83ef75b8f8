#!/usr/bin/env python3
"""The skv kernels of a rocprofv3 --stats CSV (run_kernel_stats.csv), names without their
parameter lists, with the time per compaction (the bench's compactions in the trace: warm-up +
steps + the invariant check's one, e.g. 5 for --steps 3 --warmup 1).

usage: kstats_skv.py run_kernel_stats.csv compactions [out.csv]"""
import csv
import re
import sys


def short(name):
    name = re.sub(r"^void ", "", name)
    depth, out = 0, []
    for ch in name:  # drop the parameter list (the outermost parentheses), keep template args
        if ch == "(":
            depth += 1
        if depth == 0:
            out.append(ch)
        if ch == ")":
            depth -= 1
    return "".join(out).strip()


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2])
    skv = [r for r in rows if "skv::" in r["Name"]]
    tot = sum(float(r["TotalDurationNs"]) for r in skv)
    out = [["kernel", "calls", "avg_us", "ms_per_compaction", "pct_of_skv_time"]]
    for r in sorted(skv, key=lambda r: -float(r["TotalDurationNs"])):
        t = float(r["TotalDurationNs"])
        out.append([short(r["Name"]), r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), round(t / 1e6 / n, 4),
                    round(100 * t / tot, 2)])
    out.append(["(all skv kernels)", sum(int(r["Calls"]) for r in skv), "", round(tot / 1e6 / n, 4), 100.0])
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w", newline="") as f:
            csv.writer(f).writerows(out)
    for o in out:
        print(f"{str(o[0])[:44]:44s} {str(o[1]):>6s} {str(o[2]):>10s} {str(o[3]):>9s} {str(o[4]):>6s}")


if __name__ == "__main__":
    main()
