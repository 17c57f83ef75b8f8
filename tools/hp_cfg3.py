"""General host pipeline probe: config 3 (256 streams x --run-mib MiB of variable-length records +
10 % Deletes, built by the GPU generator) in pinned host memory through skv_compact, serial (SKV_HOST_PIPE=0) against the
key-range pipeline at several part counts; wall time per call (best of 3). With SKV_HOST_TRACE=1
the library prints its host-side milestones of every call.

usage: python tools/hp_cfg3.py [--run-mib 16] [P ...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "skyvault-rs_amd"))

import torch  # noqa: E402

from skv.api import Compactor  # noqa: E402
from skv.devgen import make_cfg3_full_on_device  # noqa: E402


def main():
    args = sys.argv[1:]
    run_mib = 16
    if args and args[0] == "--run-mib":
        run_mib = int(args[1])
        args = args[2:]
    parts = [int(a) for a in args] or [0, 8, 14, 32]
    torch.cuda.init()
    dev = torch.device("cuda:0")
    runs = make_cfg3_full_on_device(dev, 0x5EEDC0DE, 256, run_mib)
    host = [r.cpu().pin_memory() for r in runs]
    del runs
    torch.cuda.empty_cache()
    streams = [(s + 1, [(r.data_ptr(), r.numel())]) for s, r in enumerate(host)]
    nbytes = sum(r.numel() for r in host)
    comp = Compactor(0)
    for P in parts:
        if P == 0:
            os.environ["SKV_HOST_PIPE"] = "0"
        else:
            os.environ.pop("SKV_HOST_PIPE", None)
            os.environ["SKV_HOST_PARTS"] = str(P)
        comp.compact_host_ptrs(streams, 4 << 20, 0)
        ts = []
        for i in range(3):
            t0 = time.perf_counter()
            comp.compact_host_ptrs(streams, 4 << 20, 0)
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        print(f"P={P} parts={comp.timings()['host_parts']} best {t * 1e3:.2f} ms = {nbytes / t / 2**30:.2f} GiB/s "
              f"(all: {', '.join(f'{x * 1e3:.1f}' for x in ts)})", flush=True)


if __name__ == "__main__":
    main()
