"""k_tile<true> (or, with a second argument 2A / 2B, k_fx_tile) phase ticks (a SKV_TILE_PROF=1 build, SKV_LIB=...): config 3 (256 streams x
--run-mib MiB, built in HBM), 1 warm-up + 3 calls of skv_compact_dev; the phase sums are printed
by skv_ctx_destroy on stderr (100 MHz ticks summed over tiles; phases: 0 segments, 1 loads,
2 merge, 3 first-per-key, 4 meta/address by position, 5 filter + scans, 6 look-back, 7 emit)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "skyvault-rs_amd"))

import torch  # noqa: E402

from skv.api import Compactor  # noqa: E402
from skv.devgen import make_cfg3_full_on_device  # noqa: E402

run_mib = int(sys.argv[1]) if len(sys.argv) > 1 else 16
dev = torch.device("cuda:0")
if len(sys.argv) > 2 and sys.argv[2] in ("2A", "2B"):  # the fused path (k_fx_tile's phases)
    from skv.devgen import make_cfg2_on_device

    runs = make_cfg2_on_device(dev, 0x5EEDC0DE, 64, 238821, 256, sys.argv[2][1])
else:
    runs = make_cfg3_full_on_device(dev, 0x5EEDC0DE, 256, run_mib)
table = [(s + 1, [(r.data_ptr(), r.numel())]) for s, r in enumerate(runs)]
comp = Compactor(0, profiling=True)
for i in range(4):
    t0 = time.perf_counter()
    r = comp.compact_dev(table, 4 << 20, 0)
    torch.cuda.synchronize()
    t = comp.timings()
    print(f"call {i}: {1e3 * (time.perf_counter() - t0):.2f} ms merge {t['merge_ms']:.2f} ms", flush=True)
    r.free()
comp.close()
