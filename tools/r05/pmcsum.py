"""Per kernel, the FETCH_SIZE / WRITE_SIZE of its last dispatch in a rocprofv3 --pmc output dir,
as HBM bytes (FETCH_SIZE x 2 per the gfx950 correction in MI355X_MICROARCH.md, units of KiB).
usage: pmcsum.py <dir> [kernel ...]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
kernels = sys.argv[2:]
last = collections.defaultdict(dict)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        d = int(r["Dispatch_Id"])
        c = r["Counter_Name"]
        if c not in last[k] or last[k][c][0] < d:
            last[k][c] = (d, float(r["Counter_Value"]))
for k in sorted(last):
    if kernels and k not in kernels and "all" not in kernels:
        continue
    cs = {c: v for c, (_, v) in last[k].items()}
    rd = cs.get("FETCH_SIZE", 0) * 2048 / 1e9
    wr = cs.get("WRITE_SIZE", 0) * 1024 / 1e9
    print(f"   {k}: read {rd:.3f} GB write {wr:.3f} GB")
