"""Staged chunk walks: parse-phase time of config 3 (256 streams x --run-mib MiB, built in HBM by
the GPU generator) under env variants, e.g.
  python tools/stage_probe.py SKV_STAGE=0 SKV_STAGE=1 SKV_STAGE=1,SKV_STAGE_DBG=1
Each variant: 1 warm-up + 3 calls of skv_compact_dev; prints the parse phase and the total."""
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
    run_mib, n_streams = 16, 256
    if args and args[0] == "--run-mib":
        run_mib, args = int(args[1]), args[2:]
    if args and args[0] == "--streams":
        n_streams, args = int(args[1]), args[2:]
    host_gen = bool(args) and args[0] == "--host-gen"  # gen.config3's runs (bench --config 3's data)
    if host_gen:
        args = args[1:]
    dev = torch.device("cuda:0")
    t0 = time.time()
    if host_gen:
        from skv import gen
        n = (run_mib << 20) // 333
        runs = []
        for s in range(n_streams):
            r = gen.var_key_run(gen.BASE_SEED + s, n, n * n_streams * 2, 256)
            runs.append(torch.from_numpy(r).to(dev))
            if s % 32 == 31:
                print(f"  generated {s + 1} runs", flush=True)
    else:
        runs = make_cfg3_full_on_device(dev, 0x5EEDC0DE, n_streams, run_mib)
    print(f"built {sum(r.numel() for r in runs) / 2**30:.2f} GiB in {time.time() - t0:.1f} s", flush=True)
    table = [(s + 1, [(r.data_ptr(), r.numel())]) for s, r in enumerate(runs)]
    comp = Compactor(0, profiling=True)
    for v in args or ["SKV_STAGE=1"]:
        env = dict(kv.split("=") for kv in v.split(","))
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        res = []
        for i in range(4):
            r = comp.compact_dev(table, 4 << 20, 0)
            r.free()
            t = comp.timings()
            if i:
                res.append((t["parse_ms"], t["total_ms"]))
            span = t["span_parse"]
        for k, o in old.items():
            if o is None:
                os.environ.pop(k)
            else:
                os.environ[k] = o
        print(f"{v:40s} parse {min(p for p, _ in res):7.2f} ms  total {min(t for _, t in res):7.2f} ms"
              f"  span_parse {span:#x}", flush=True)


if __name__ == "__main__":
    main()
