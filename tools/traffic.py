"""Per-launch HBM traffic of each skv kernel from two rocprofv3 --pmc passes (tools/gpu_pmc.sh with
PMC_GROUPS="FETCH_SIZE WRITE_SIZE"), corrected as MI355X_MICROARCH.md § HBM prescribes for gfx950:
FETCH_SIZE (KiB) counts half the bytes of wide streaming reads -> x2; WRITE_SIZE (KiB) is exact for
16 B/lane stores. Uses the LAST dispatch of each kernel (the timed step of bench.py --steps 1).

usage: python tools/traffic.py gpurun_out/pmc [profiles/traffic_latest.json]
"""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]
out = sys.argv[2] if len(sys.argv) > 2 else None
last = collections.defaultdict(dict)  # kernel -> counter -> value of its last dispatch
for f in sorted(glob.glob(f"{root}/g*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        last[k][r["Counter_Name"]] = (int(r["Dispatch_Id"]), float(r["Counter_Value"]))

kernels = {}
for k, cs in last.items():
    if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
        continue
    rd = cs["FETCH_SIZE"][1] * 1024 * 2
    wr = cs["WRITE_SIZE"][1] * 1024
    kernels[k] = {"read_bytes": int(rd), "write_bytes": int(wr), "hbm_bytes": int(rd + wr)}
for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["hbm_bytes"])[:20]:
    print(f"{k[:48]:48s} read={v['read_bytes'] / 1e9:8.3f} GB write={v['write_bytes'] / 1e9:8.3f} GB")
g = kernels.get("skv::k_gather")
doc = {
    "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, last dispatch per kernel",
    "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), WRITE_SIZE x1; KiB -> bytes",
    "gather_hbm_bytes_per_launch": g["hbm_bytes"] if g else None,
    "kernels": kernels,
}
if out:
    with open(out, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    print("wrote", out)
