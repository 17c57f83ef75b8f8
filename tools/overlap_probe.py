"""Back-to-back config-2A compactions on one GPU: one ctx (each call waits for the previous) vs two
ctxs driven from two host threads (one call's splitter phase and host gaps beside the other's tile
phase). Prints ms per compaction for each. Inputs are built once in HBM and shared (read-only)."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "skyvault-rs_amd"))

import torch  # noqa: E402

from skv._abi import StreamArgs  # noqa: E402
from skv.api import Compactor  # noqa: E402
from skv.devgen import make_cfg2_on_device  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 40
dev = torch.device("cuda:0")
runs = make_cfg2_on_device(dev, 0x5EEDC0DE, 64, 238821, 256, "A")
table = StreamArgs([(s + 1, [(r.data_ptr(), r.numel())]) for s, r in enumerate(runs)], device=True)
in_bytes = sum(r.numel() for r in runs)
cs = [Compactor(0) for _ in range(3)]


def loop(c, n):
    for _ in range(n):
        c.compact_dev(table, 4 << 20, 0).free()


for c in cs:
    loop(c, 3)
torch.cuda.synchronize()
for nctx in (1, 2, 3, 1, 2):
    th = [threading.Thread(target=loop, args=(cs[i], K // nctx)) for i in range(nctx)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n = (K // nctx) * nctx
    print(f"{nctx} ctx: {dt / n * 1e3:.3f} ms per compaction, {in_bytes * n / dt / 2**30:.1f} GiB/s", flush=True)
