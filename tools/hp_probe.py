"""Pipelined host path probe: config 2A in pinned host memory through skv_compact, a few calls per
part count (SKV_HOST_PARTS), wall time per call. Run under rocprofv3 --kernel-trace
--memory-copy-trace to see the H2D / kernel / D2H overlap per part.

usage: python tools/hp_probe.py [P ...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "skyvault-rs_amd"))

import torch  # noqa: E402

from skv.api import Compactor  # noqa: E402
from skv.devgen import make_cfg2_on_device  # noqa: E402


def main():
    parts = [int(a) for a in sys.argv[1:]] or [15]
    torch.cuda.init()
    dev = torch.device("cuda:0")
    runs = make_cfg2_on_device(dev, 1, 64, 238821, 256, "A")
    host = [r.cpu().pin_memory() for r in runs]
    del runs
    torch.cuda.empty_cache()
    streams = [(s + 1, [(r.data_ptr(), r.numel())]) for s, r in enumerate(host)]
    nbytes = sum(r.numel() for r in host)
    comp = Compactor(0)
    for P in parts:
        os.environ["SKV_HOST_PARTS"] = str(P)
        comp.compact_host_ptrs(streams, 4 << 20, 0)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            comp.compact_host_ptrs(streams, 4 << 20, 0)
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        print(f"P={P} parts={comp.timings()['host_parts']} best {t * 1e3:.2f} ms "
              f"{nbytes / t / 2**30:.2f} GiB/s  all {[round(x * 1e3, 1) for x in ts]}", flush=True)
    # the copy engines alone: H2D, D2H, both at once (one 4 GiB pinned buffer each way)
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)),
                     ("d2h", lambda: h.copy_(d, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        print(f"{name} alone {nbytes / t / 1e9:.1f} GB/s", flush=True)
    half = nbytes // 2
    d2 = torch.empty(half, dtype=torch.uint8, device=dev)
    h2 = torch.empty(half, dtype=torch.uint8).pin_memory()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(s1):
        d[:half].copy_(h[:half], non_blocking=True)
    with torch.cuda.stream(s2):
        h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    print(f"h2d+d2h concurrent {half / 1e9:.2f} GB each way: {t * 1e3:.1f} ms, {2 * half / t / 1e9:.1f} GB/s total",
          flush=True)
    comp.close()


if __name__ == "__main__":
    main()
