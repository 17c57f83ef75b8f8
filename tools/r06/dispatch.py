#!/usr/bin/env python3
"""Per-dispatch summary of a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv) for the skv kernels,
restricted to the bench's TIMED compactions (measurement hygiene).

The bench runs W warm-up compactions, K timed ones and one invariant-check call (bench.py
timed_loop / check_invariants). Compactions are told apart by the first kernel of each call (the
kernel named by --first, default: the first skv kernel of the trace): dispatch i starts a new
compaction when it is that kernel (every m-th occurrence when each call launches it m times,
m = its count / (W + K + 1)). The first W compactions and everything after the K-th timed one are
dropped, so per-kernel totals can never exceed the traced ms_per_step.

usage: dispatch.py run_kernel_trace.csv W K [--first NAME] [--out stats.csv] [--top N]"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    name = re.sub(r"^void ", "", name)
    depth, out = 0, []
    for ch in name:
        if ch == "(":
            depth += 1
        if depth == 0:
            out.append(ch)
        if ch == ")":
            depth -= 1
    return re.sub(r"^skv::", "", "".join(out).strip())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("W", type=int)
    ap.add_argument("K", type=int)
    ap.add_argument("--first", default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--dispatches", default=None, help="write every timed dispatch of this kernel")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            if "skv::" not in r["Kernel_Name"]:
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    first = a.first or rows[0][2]
    # a call that launches its first kernel m times (config 5: k_run_info twice) starts at every m-th
    # occurrence; the bench's calls are W warm-ups, K timed and one invariant check
    m = 1 if a.first else max(1, sum(1 for r in rows if r[2] == first) // (a.W + a.K + 1))
    calls, cur, seen = [], None, 0
    for s, e, n in rows:
        if n == first:
            seen += 1
        if (n == first and (seen - 1) % m == 0) or cur is None:
            cur = []
            calls.append(cur)
        cur.append((s, e, n))
    timed = calls[a.W:a.W + a.K]
    span = [(c[0][0], max(e for _, e, _ in c)) for c in timed]
    agg = defaultdict(lambda: [0, 0, 0, 1 << 62])  # calls, total ns, max, min
    for c in timed:
        for s, e, n in c:
            g = agg[n]
            g[0] += 1
            g[1] += e - s
            g[2] = max(g[2], e - s)
            g[3] = min(g[3], e - s)
    tot = sum(g[1] for g in agg.values())
    print(f"compactions in trace {len(calls)}, timed {len(timed)} (W={a.W} dropped, the rest after K dropped); "
          f"first kernel {first}")
    print(f"first->last kernel span per timed compaction: "
          f"{sum(e - s for s, e in span) / len(span) / 1e6:.4f} ms avg")
    out = [["kernel", "calls", "avg_us", "min_us", "max_us", "ms_per_compaction", "pct"]]
    for n, g in sorted(agg.items(), key=lambda x: -x[1][1]):
        out.append([n, g[0], round(g[1] / g[0] / 1e3, 1), round(g[3] / 1e3, 1), round(g[2] / 1e3, 1),
                    round(g[1] / 1e6 / len(timed), 4), round(100 * g[1] / tot, 2)])
    out.append(["(all skv kernels)", sum(g[0] for g in agg.values()), "", "", "", round(tot / 1e6 / len(timed), 4), 100.0])
    if a.out:
        with open(a.out, "w", newline="") as f:
            csv.writer(f).writerows(out)
    for o in out:
        print(f"{str(o[0])[:40]:40s} {str(o[1]):>6s} {str(o[2]):>9s} {str(o[3]):>9s} {str(o[4]):>9s} {str(o[5]):>9s} {str(o[6]):>6s}")
    if a.dispatches:
        print(f"-- every dispatch of {a.dispatches} (all compactions, c = compaction index, timed from {a.W})")
        for ci, c in enumerate(calls):
            for s, e, n in c:
                if n == a.dispatches:
                    print(f"c={ci} start={(s - rows[0][0]) / 1e6:.3f} ms dur={(e - s) / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
