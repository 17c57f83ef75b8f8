"""Per-launch HBM traffic of each skv kernel of ONE bench config from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE: separate runs, kernel-trace only), corrected as MI355X_MICROARCH.md § HBM
prescribes for gfx950: FETCH_SIZE (KiB) counts half the bytes of wide streaming reads -> x2;
WRITE_SIZE (KiB) is exact for 16 B/lane stores. Uses the LAST dispatch of each kernel (the timed
step of bench.py --steps 1).

The traffic file is keyed by config and kernel ({"configs": {"2A": {"kernels": {...}}}}) so that
bench.py reports a config's own counters for its own dominant kernel, never another config's.

Per call: every dispatch of the TIMED compaction (the run's calls are warm-up,
timed, invariant check: --steps 1 --warmup 1 -> 3 calls; a call starts at the kernel of the run's
first dispatch, or at every m-th occurrence of it when a call launches it m times) summed per kernel
and over all kernels -> "call": {"read_bytes", "write_bytes", "hbm_bytes", "launches"}.

usage: python tools/traffic.py <pmc dir with g*/...counter_collection.csv> <config> [traffic.json] [calls]
"""
import collections
import csv
import glob
import json
import os
import sys

root, config = sys.argv[1], sys.argv[2]
out = sys.argv[3] if len(sys.argv) > 3 else None
n_calls = int(sys.argv[4]) if len(sys.argv) > 4 else 3
TIMED = 1  # the call after the one warm-up
last = collections.defaultdict(dict)  # kernel -> counter -> (dispatch, value) of its last dispatch
per_call = collections.defaultdict(lambda: collections.defaultdict(float))  # counter -> kernel -> timed-call sum
launches = collections.Counter()  # kernel -> dispatches in the timed call (from the first counter's run)
files = sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True))
for fi, f in enumerate(files):
    rows = collections.defaultdict(dict)  # dispatch -> (kernel, {counter: value}) of this pass
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        d = int(r["Dispatch_Id"])
        c = r["Counter_Name"]
        v = float(r["Counter_Value"])
        if c not in last[k] or last[k][c][0] <= d:
            last[k][c] = (d, v)
        rows[d].setdefault("k", k)
        rows[d][c] = rows[d].get(c, 0.0) + v
    seq = [(d, rows[d]) for d in sorted(rows) if rows[d]["k"].startswith("skv::")]
    if not seq:
        continue
    first = seq[0][1]["k"]
    m = max(1, sum(1 for _, x in seq if x["k"] == first) // n_calls)
    call, seen = -1, 0
    for d, x in seq:
        if x["k"] == first:
            if seen % m == 0:
                call += 1
            seen += 1
        if call != TIMED:
            continue
        for c, v in x.items():
            if c != "k":
                per_call[c][x["k"]] += v
        if fi == 0:
            launches[x["k"]] += 1

kernels = {}
for k, cs in last.items():
    if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
        continue
    rd = cs["FETCH_SIZE"][1] * 1024 * 2
    wr = cs["WRITE_SIZE"][1] * 1024
    kernels[k] = {"read_bytes": int(rd), "write_bytes": int(wr), "hbm_bytes": int(rd + wr)}
rd_c = sum(per_call["FETCH_SIZE"].values()) * 1024 * 2
wr_c = sum(per_call["WRITE_SIZE"].values()) * 1024
call = {"read_bytes": int(rd_c), "write_bytes": int(wr_c), "hbm_bytes": int(rd_c + wr_c),
        "launches": sum(launches.values()),
        "kernels": {k: int(per_call["FETCH_SIZE"].get(k, 0) * 2048 + per_call["WRITE_SIZE"].get(k, 0) * 1024)
                    for k in set(per_call["FETCH_SIZE"]) | set(per_call["WRITE_SIZE"])}}
print(f"timed call: {call['launches']} launches, read={rd_c / 1e9:.3f} GB write={wr_c / 1e9:.3f} GB")
for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["hbm_bytes"])[:20]:
    print(f"{k[:48]:48s} read={v['read_bytes'] / 1e9:8.3f} GB write={v['write_bytes'] / 1e9:8.3f} GB")
if out:
    doc = {}
    if os.path.exists(out):
        doc = json.load(open(out))
    if "configs" not in doc:  # an older single-config file: start over, keyed by config
        doc = {}
    doc["source"] = "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, last dispatch per kernel"
    doc["correction"] = "FETCH_SIZE x2 (gfx950 wide streaming reads), WRITE_SIZE x1; KiB -> bytes"
    doc.setdefault("configs", {})[config] = {
        "pmc_passes": "bench.py --config %s --steps 1 --warmup 1: rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE" % config,
        "kernels": kernels, "call": call}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    print("wrote", out, "config", config)
