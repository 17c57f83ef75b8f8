"""Random-shape sweep of the device path (skv_compact with the pipelines off: stage -> compact_device
-> copy) against the oracle: fixed or variable records, Deletes, member runs, both flags, run sizes
from one record to unbounded, fan-in from 1 to 40 streams and, one seed in eight, 1,600-2,400 tiny
streams (the record sort past 1,536).
usage: python tools/r05/dev_fuzz.py [first_seed] [n_seeds]"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "skyvault-rs_amd"), os.path.join(ROOT, "oracle")]

import torch  # noqa: E402

from skv import _abi  # noqa: E402
from skv import format as fmt  # noqa: E402
from skv.api import Compactor  # noqa: E402
from test_gpu_parity import _diff, _run_both  # noqa: E402

torch.cuda.init()
dev = Compactor(0)
os.environ["SKV_HOST_PIPE"] = "0"
a = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 400
bad = piped = 0
for seed in range(a, a + n):
    rng = random.Random(6271 * seed + 17)
    flags = rng.choice([0, 0, _abi.SKV_DROP_TOMBSTONES])
    fixed = rng.random() < 0.4
    vlen = rng.choice([0, 8, 40, 200])
    space = rng.choice([2000, 20000, 200000])
    streams = []
    wide = rng.random() < 0.125
    for s in range(rng.randint(1600, 2400) if wide else rng.randint(1, 40)):
        ids = sorted(rng.sample(range(space), min(rng.randint(0, 12) if wide else rng.randint(0, 3000), space)))
        if not ids:
            continue
        nm = rng.choice([1, 1, 1, 3])
        cuts = sorted(rng.sample(range(1, len(ids)), min(nm - 1, len(ids) - 1))) if len(ids) > 1 else []
        bounds = [0] + cuts + [len(ids)]
        members = []
        for x, y in zip(bounds, bounds[1:]):
            ops = []
            for i in ids[x:y]:
                key = f"k{i:09d}" if fixed else f"k{i:09d}" + "x" * (i % 13)
                if not fixed and rng.random() < 0.1:
                    ops.append(fmt.delete(key))
                else:
                    ops.append(fmt.put(key, bytes([i & 0xFF]) * (vlen if fixed else (i * 7) % (vlen + 1))))
            members.append(fmt.encode_run(ops))
        streams.append((s + 1, members))
    if not streams:
        continue
    max_size = rng.choice([1, 100, 1000, 4096, 1 << 20, 1 << 62])
    exp, got = _run_both(dev, streams, max_size, flags)
    piped += dev.timings()["path"] == 3  # (fused)
    if exp != got:
        bad += 1
        print(f"seed {seed}: MISMATCH {_diff(exp, got)[:300]}", flush=True)
    if seed % 50 == 0:
        print(f"seed {seed} done, {bad} bad, {piped} fused", flush=True)
print(f"{n} seeds from {a}: {bad} mismatches, {piped} on the fused path", flush=True)
dev.close()
sys.exit(1 if bad else 0)
