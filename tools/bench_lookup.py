#!/usr/bin/env python3
"""Batched run lookups (skv_search_run) on one 4 MiB run of config-2 records (16 B hex keys,
256 B values, ~14.9 k records), 2^20 keys per call (half present, half absent). Reports
lookups/s of the whole call (host run + keys staged to HBM, outcomes back to host)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "skyvault-rs_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from skv import gen  # noqa: E402
from skv.api import Compactor  # noqa: E402

torch.cuda.init()
n = (4 << 20) // 281
ids = gen.unique_sorted_u64(7, n)
run = gen.hex_key_run(7, n, 256).tobytes()
keys = gen.hex16(ids)
rng = np.random.default_rng(1)
q = 1 << 20
present = keys[rng.integers(0, n, q // 2)]
absent = gen.hex16(rng.integers(0, 2 ** 63, q // 2, dtype=np.uint64))
qs = [bytes(x) for x in np.concatenate([present, absent])]
c = Compactor(0, profiling=True)
c.search_run(run, qs[:1000])
ts = []
for _ in range(3):
    t0 = time.perf_counter()
    res = c.search_run(run, qs)
    ts.append(time.perf_counter() - t0)
found = sum(1 for r in res if r[0] == "found")
t = min(ts)
print(json.dumps({"lookups_per_s": round(q / t), "ms_per_call": round(t * 1e3, 2), "keys": q, "records": n,
                  "found": found, "path": "bsearch" if c.timings()["path"] == 2 else "scan"}))
