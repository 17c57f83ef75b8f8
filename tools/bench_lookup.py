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
qk = np.ascontiguousarray(np.concatenate([present, absent]))  # (q, 16) uint8, all 16 B keys
offs = np.arange(q + 1, dtype=np.uint64) * 16
out = np.zeros(q, dtype=np.dtype([("kind", np.uint32), ("panic", np.uint32), ("off", np.uint64), ("len", np.uint64)]))
c = Compactor(0, profiling=True)
rb = np.frombuffer(run, dtype=np.uint8)
import ctypes as C  # noqa: E402


def call():
    rc = c.lib.skv_search_run(c.ctx, C.c_void_p(rb.ctypes.data), len(run), C.c_void_p(qk.ctypes.data),
                              C.c_void_p(offs.ctypes.data), q, C.c_void_p(out.ctypes.data))
    assert rc == 0, rc


call()
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    call()
    ts.append(time.perf_counter() - t0)
t = min(ts)
tm = c.timings()
print(json.dumps({"lookups_per_s": round(q / t), "ms_per_call": round(t * 1e3, 3), "device_ms": round(tm["total_ms"], 3),
                  "keys": q, "records": n, "found": int((out["kind"] == 1).sum()),
                  "path": "bsearch" if tm["path"] == 2 else "scan",
                  "note": "whole skv_search_run call: 4 MiB run + 16 MiB of keys staged H2D, outcomes D2H"}))
