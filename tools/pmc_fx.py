"""Summarise tools/gpu_pmc_fx.sh output: per library, the counters of the last dispatch of each
kernel named on the command line (default skv::k_fx_tile).
usage: python tools/pmc_fx.py gpurun_out/pmcfx [kernel ...]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
kernels = sys.argv[2:] or ["skv::k_fx_tile"]
for libdir in sorted(glob.glob(os.path.join(root, "*/"))):
    last = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(libdir, "g*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            d = int(r["Dispatch_Id"])
            c = r["Counter_Name"]
            if c not in last[k] or last[k][c][0] < d:
                last[k][c] = (d, float(r["Counter_Value"]))
    for k in kernels:
        cs = {c: v for c, (_, v) in last.get(k, {}).items()}
        if not cs:
            continue
        line = " ".join(f"{c}={v:.4g}" for c, v in sorted(cs.items()))
        print(f"{os.path.basename(libdir.rstrip('/'))} {k}: {line}")
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            print(f"   HBM read ~{cs['FETCH_SIZE'] * 2048 / 1e9:.3f} GB (x2 corrected), write {cs['WRITE_SIZE'] * 1024 / 1e9:.3f} GB")
