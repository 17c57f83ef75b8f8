"""Random WAL flushes (SKV_SPLIT_BY_TABLE) through the device path and the split against the
oracle: 1-300 sorted runs, table ids incl. negative ones, a few non-canonical prefixes ("007.",
"-0.", no '.': JobError::InvalidInput), Puts and Deletes, value sizes, max_run_size from one record
to unbounded (the exactly-one-run rule drops tables). Unsorted WAL runs are left out: their failed-
send window is a documented race.
usage: python tools/r05/wal_fuzz.py [first_seed] [n_seeds]"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "skyvault-rs_amd"), os.path.join(ROOT, "oracle")]

import torch  # noqa: E402

from skv import _abi  # noqa: E402
from skv import format as fmt  # noqa: E402
from skv.api import Compactor, compact_split  # noqa: E402
import pyoracle  # noqa: E402
from test_gpu_parity import _diff, _norm, _run_both  # noqa: E402

torch.cuda.init()
dev = Compactor(0)
cs = [Compactor(0) for _ in range(4)]
a = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
bad = 0
BAD_PREFIXES = ["007.", "-0.", "12x", "+5.", ""]
for seed in range(a, a + n):
    rng = random.Random(4099 * seed + 5)
    n_tables = rng.choice([1, 3, 20, 64])
    tables = [str(t) for t in rng.sample(range(-50, 10000), n_tables)]
    p_bad = rng.choice([0, 0, 0, 0.001, 0.01])
    vmax = rng.choice([0, 8, 64])
    runs = []
    for r in range(rng.randint(1, 300)):
        keys = set()
        for _ in range(rng.randint(1, 60)):
            pre = rng.choice(BAD_PREFIXES) if rng.random() < p_bad else rng.choice(tables) + "."
            keys.add(pre + f"{rng.randrange(10**6):06d}")
        ops = []
        for k in sorted(keys):
            if rng.random() < 0.1:
                ops.append(fmt.delete(k))
            else:
                ops.append(fmt.put(k, bytes([rng.randrange(256)]) * rng.randint(0, vmax)))
        runs.append(fmt.encode_run(ops))
    streams = [(i + 1, [r]) for i, r in enumerate(runs)]
    max_size = rng.choice([1, 200, 4096, 1 << 20, 1 << 62])
    exp, got = _run_both(dev, streams, max_size, _abi.SKV_SPLIT_BY_TABLE)
    if exp != got:
        bad += 1
        print(f"seed {seed}: device MISMATCH {_diff(exp, got)[:300]}", flush=True)
    try:
        r2, info = compact_split(cs, streams, max_size, _abi.SKV_SPLIT_BY_TABLE, with_info=True)
        got2 = ("ok", _norm(r2), info["dropped_tables"])
    except _abi.RunError as e:
        got2 = ("err", e.code, e.message)
    if exp != got2:
        bad += 1
        print(f"seed {seed}: split MISMATCH {_diff(exp, got2)[:300]}", flush=True)
    if seed % 50 == 0:
        print(f"seed {seed} done, {bad} bad", flush=True)
print(f"{n} seeds from {a}: {bad} mismatches", flush=True)
sys.exit(1 if bad else 0)
