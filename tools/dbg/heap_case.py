"""Diagnostic: one heap-order DROP case from test_drop_tombstones_with_unsorted_stream_matches_oracle."""
import os, sys, random
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, p) for p in ("tests", "oracle", "skyvault-rs_amd")]
import torch
torch.cuda.init()
from skv import format as fmt, _abi
from skv.api import Compactor
import pyoracle
os.environ["SKV_HEAP_DEBUG"] = "1"
r = random.Random(31)
cases = []
for trial in range(150):
    streams = []
    for s in range(r.randint(1, 6)):
        keys = sorted({f"k{r.randrange(60):03d}" for _ in range(r.randint(0, 25))})
        for _ in range(r.randint(0, 2)):
            if len(keys) > 1:
                i = r.randrange(len(keys) - 1)
                keys[i], keys[i + 1] = keys[i + 1], keys[i]
        ops = [fmt.delete(k) if r.random() < 0.5 else fmt.put(k, bytes([r.randrange(256)]) * r.randrange(4)) for k in keys]
        run = fmt.encode_run(ops)
        if r.random() < 0.15 and len(run) > 2:
            run = run[: r.randrange(1, len(run))]
        members = [run] if r.random() < 0.8 else [run, fmt.encode_run([fmt.put("zz%d" % s, b"m")])]
        streams.append((s * 7 + 1, members))
    cases.append(streams)
c = Compactor(0)
for i in (3,):
    try:
        got = c.compact(cases[i], 4 << 20, 1)
        print("ok", len(got))
    except _abi.RunError as e:
        print("err", e)
good = fmt.encode_run([fmt.put("1.a", b"x"), fmt.put("2.b", b"y")])
bad_key = fmt.encode_run([fmt.put("1.0", b"x"), fmt.put("nodot", b"y"), fmt.put("3.z", b"y")])
unsorted = fmt.encode_run([fmt.put("2.c", b"u"), fmt.put("1.b", b"u"), fmt.put("1.d", b"u"), fmt.put("3.a", b"u")])
for streams in ([(2, [bad_key]), (1, [good[:-3]])], [(3, [unsorted]), (1, [good])]):
    try:
        got = c.compact(streams, 4 << 20, 2)
        print("ok", [(r.table_id, r.data) for r in got])
    except _abi.RunError as e:
        print("err", e)
    try:
        print("oracle", [(r.table_id, r.data) for r in pyoracle.compact(streams, 4 << 20, 2)])
    except _abi.RunError as e:
        print("oracle err", e)
