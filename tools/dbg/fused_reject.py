"""Debug helper: replay test_fused_random_shapes' trials and print the fused reject reason."""
import os, random, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "skyvault-rs_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "oracle"))
import torch
from skv import _abi
from skv.api import Compactor
from test_gpu_fused import _run, KiB, MiB
torch.cuda.init()
dev = Compactor(0, profiling=True)
r = random.Random(1234)
for trial in range(40):
    K = r.choice([2, 5, 8, 11, 16])
    V = r.randint(max(0, 32 - 9 - K), 120)
    k = r.choice([1, 2, 3, 7, 16, 64, 130])
    n = r.randint(1, 3000)
    uni = r.choice([0, k * n, max(1, n // 2)])
    if K <= 3:
        uni = min(uni or 16 ** K, 16 ** K)
    if uni:
        n = min(n, uni)
    max_size = r.choice([0, 9 + K + V, 2 * (9 + K + V) + 1, 5000, 64 * KiB, 4 * MiB])
    streams = [(r.randrange(-10**12, 10**12) * 1000 + s, [_run(trial * 1000 + s, n, K, V, uni)]) for s in range(k)]
    try:
        dev.compact(streams, max_size, 0)
    except Exception as e:
        print(trial, "err", e)
    t = dev.timings()
    if t["path"] != _abi.PATH_FUSED:
        print(trial, K, V, k, n, uni, max_size, "path", t["path"], "reject", hex(t["fused_reject"]))
