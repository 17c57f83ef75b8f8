"""Debug: the oversized last run of a general-pipeline part (test_general_pipeline_one_record_runs_
and_large_records at max 900). Runs the same inputs (1) whole, serial (SKV_HOST_PIPE=0), and (2) as
key-range sub-jobs re-encoded as runs, each with the previous range's last output run as an extra
stream at the lowest SeqNo -- what a part does, without part mode -- checking every output run's
size against max and the bytes against the oracle."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "skyvault-rs_amd"), os.path.join(ROOT, "oracle")]
os.environ["SKV_HOST_PIPE"] = "0"
from skv import format as fmt  # noqa: E402
from skv.api import Compactor  # noqa: E402
import pyoracle  # noqa: E402

rng = random.Random(17)
streams, ops_by_stream = [], []
for s in range(5):
    ids = sorted(rng.sample(range(3000), 400))
    ops = [fmt.put(f"r{i:06d}", bytes([s]) * rng.choice([10, 900, 3000])) for i in ids]
    ops_by_stream.append(ops)
    streams.append((s + 1, [fmt.encode_run(ops)]))
c = Compactor(0)
mx = 900


def check(sts, what):
    got = c.compact(sts, mx, 0)
    exp = pyoracle.compact(sts, mx, 0)
    bad = [i for i, r in enumerate(got) if len(r.data) > mx and r.stats.put_count + r.stats.delete_count > 1]
    same = [r.data for r in got] == [r.data for r in exp]
    print(f"{what}: runs {len(got)} vs {len(exp)}, equal {same}, oversized {bad[:5]} t={c.timings()['path']}",
          flush=True)
    return got


check(streams, "whole")
keys = sorted({op[1] for ops in ops_by_stream for op in ops})
cuts = [keys[p * len(keys) // 6] for p in range(1, 6)] + [None]
lo = None
carry = None
for p, hi in enumerate(cuts):
    sts = []
    for s, ops in enumerate(ops_by_stream):
        sel = [op for op in ops if (lo is None or op[1] >= lo) and (hi is None or op[1] < hi)]
        if sel:
            sts.append((s + 1, [fmt.encode_run(sel)]))
    if carry is not None:
        sts.append((-100, [carry]))
    got = check(sts, f"range {p}")
    carry = got[-1].data if got else None
    lo = hi
