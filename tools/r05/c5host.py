"""Config-5 host entry probe: 10^6 WAL runs in pinned host memory through skv_compact, with the
library's host trace on stderr (SKV_HOST_TRACE=1). usage: c5host.py [n_streams] [table|args]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "skyvault-rs_amd"))
import numpy as np
import torch

from skv import _abi
from skv._abi import StreamArgs
from skv.api import Compactor
from skv.devgen import make_cfg5_on_device

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
mode = sys.argv[2] if len(sys.argv) > 2 else "table"
torch.cuda.init()
buf = make_cfg5_on_device(torch.device("cuda", 0), 0x5EEDC0DE + 5, n)
h = buf.cpu().pin_memory()
del buf
rl = h.shape[1]
if mode == "table":
    sa = _abi.stream_table(np.arange(1, n + 1), h.data_ptr() + rl * np.arange(n, dtype=np.uint64), np.full(n, rl))
else:
    sa = StreamArgs([(s + 1, [(h.data_ptr() + s * rl, rl)]) for s in range(n)], device=True)
c = Compactor(0)
for rep in range(3):
    t0 = time.perf_counter()
    hr = c.compact_host(sa, 1 << 62, _abi.SKV_SPLIT_BY_TABLE)
    dt = time.perf_counter() - t0
    t = c.timings()
    print(f"rep {rep}: {dt * 1e3:.1f} ms, {h.numel() / dt / 2**30:.2f} GiB/s, parts {t['host_parts']}, runs {hr.n_runs}",
          file=sys.stderr, flush=True)
    hr.free()
