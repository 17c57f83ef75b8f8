"""Random-shape sweep of skv_compact_split against the oracle (the body of
tests/test_gpu_shard_split.py::test_split_random_shapes over more seeds).
usage: python tools/r05/split_fuzz.py [first_seed] [n_seeds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "skyvault-rs_amd"), os.path.join(ROOT, "oracle")]

import torch  # noqa: E402

import test_gpu_shard_split as T  # noqa: E402
from skv.api import Compactor  # noqa: E402

torch.cuda.init()
cs = [Compactor(0) for _ in range(8)]
a = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
bad = 0
for seed in range(a, a + n):
    try:
        T.test_split_random_shapes(cs, seed)
    except AssertionError as e:
        bad += 1
        print(f"seed {seed}: MISMATCH {str(e)[:300]}", flush=True)
    if seed % 50 == 0:
        print(f"seed {seed} done, {bad} bad", flush=True)
print(f"{n} seeds from {a}: {bad} mismatches", flush=True)
for c in cs:
    c.close()
sys.exit(1 if bad else 0)
