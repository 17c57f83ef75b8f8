"""Per-launch HBM traffic of each skv kernel of ONE bench config from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE: separate runs, kernel-trace only), corrected as MI355X_MICROARCH.md § HBM
prescribes for gfx950: FETCH_SIZE (KiB) counts half the bytes of wide streaming reads -> x2;
WRITE_SIZE (KiB) is exact for 16 B/lane stores. Uses the LAST dispatch of each kernel (the timed
step of bench.py --steps 1).

The traffic file is keyed by config and kernel ({"configs": {"2A": {"kernels": {...}}}}) so that
bench.py reports a config's own counters for its own dominant kernel, never another config's.

usage: python tools/traffic.py <pmc dir with g*/...counter_collection.csv> <config> [traffic.json]
"""
import collections
import csv
import glob
import json
import os
import sys

root, config = sys.argv[1], sys.argv[2]
out = sys.argv[3] if len(sys.argv) > 3 else None
last = collections.defaultdict(dict)  # kernel -> counter -> (dispatch, value) of its last dispatch
files = sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True))
for f in files:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        d = int(r["Dispatch_Id"])
        c = r["Counter_Name"]
        if c not in last[k] or last[k][c][0] <= d:
            last[k][c] = (d, float(r["Counter_Value"]))

kernels = {}
for k, cs in last.items():
    if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
        continue
    rd = cs["FETCH_SIZE"][1] * 1024 * 2
    wr = cs["WRITE_SIZE"][1] * 1024
    kernels[k] = {"read_bytes": int(rd), "write_bytes": int(wr), "hbm_bytes": int(rd + wr)}
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
        "kernels": kernels}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    print("wrote", out, "config", config)
