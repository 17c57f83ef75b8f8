"""Span parse debug: a small config-3 call (host-generated variable-length runs) with
SKV_SPAN_DBG=1 (the span kernels printf their first failing lanes), checked against the oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "skyvault-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import torch  # noqa: E402

torch.cuda.init()
from skv import gen  # noqa: E402
from skv.api import Compactor  # noqa: E402

import pyoracle  # noqa: E402

os.environ["SKV_SPAN_DBG"] = "1"
streams = gen.config3(n_streams=int(sys.argv[1]) if len(sys.argv) > 1 else 4,
                      run_bytes=int(sys.argv[2]) if len(sys.argv) > 2 else 200_000)
c = Compactor(0, profiling=True)
got = c.compact(streams, 64 * 1024, 0)
t = c.timings()
print("span_parse", hex(t["span_parse"]), "parse_ms", t["parse_ms"], flush=True)
for _ in range(2):
    c.compact(streams, 64 * 1024, 0)
    t = c.timings()
    print("span_parse", hex(t["span_parse"]), "parse_ms", t["parse_ms"], flush=True)
if len(sys.argv) <= 3:
    exp = pyoracle.compact(streams, 64 * 1024, 0)
    print("equal", [r.data for r in got] == [r.data for r in exp])
c.close()
