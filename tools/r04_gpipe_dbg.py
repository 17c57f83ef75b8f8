"""Debug: the general pipeline on test_general_pipeline_one_record_runs_and_large_records' input,
per-part runs printed by the library (SKV_GPIPE_DEBUG=1)."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "skyvault-rs_amd"), os.path.join(ROOT, "oracle")]
os.environ["SKV_HOST_PIPE_MIN"] = "0"
os.environ["SKV_HOST_PARTS"] = "6"
os.environ["SKV_GPIPE_DEBUG"] = "1"
from skv import format as fmt  # noqa: E402
from skv.api import Compactor  # noqa: E402

rng = random.Random(17)
streams = []
for s in range(5):
    ids = sorted(rng.sample(range(3000), 400))
    streams.append((s + 1, [fmt.encode_run([fmt.put(f"r{i:06d}", bytes([s]) * rng.choice([10, 900, 3000])) for i in ids])]))
c = Compactor(0)
for mx in (1, 900, 2500, 8000):
    print("max", mx, flush=True)
    try:
        c.compact(streams, mx, 0)
        print("ok", c.timings()["host_parts"], flush=True)
    except Exception as e:
        print("ERR", e, flush=True)
