#!/usr/bin/env python3
"""Compaction throughput on MI355X — BASELINE.json's metric:
"compaction GiB/s of input run bytes merged (device-resident), 1/2/4/8 GPU".

Workload (BASELINE.json configs[1], SURVEY.md §8d config 2 variant A): a 64-way L0->L1
compaction of 64 streams x 1 run x 238,821 records (16 B hex keys, 256 B values, 281 B per
record, 67,108,702 B per run, 4.0 GiB total), max run size 4 MiB, no tombstones. One step
= one whole compaction (decode, merge, dedup, greedy split, stats, output bytes) with the
inputs already resident in HBM. At N GPUs every rank runs its own independent compaction
(distinct seeds; BASELINE config 4 at N=8): weak scaling, no collective on the data path.

Prints ONE JSON line on rank 0 with `roofline` (the gather kernel: algorithmic bytes / its
HIP-event-timed duration on the library stream) and `cpu_baseline` (the C restatement in
oracle/, faithful shape, 1 core, on a bounded sample of the same workload).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "skyvault-rs_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "compaction GiB/s of input run bytes merged (device-resident), 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
MAX_RUN = 4 * 1024 * 1024
# the dominant kernel of each device path (skv_timings.path) and what its bytes count
HOT_KERNEL = {1: "k_gather", 2: "k_gather", 3: "k_fx_tile"}
PATH_NAMES = {1: "general", 2: "fixed", 3: "fused"}
GiB = float(1 << 30)


def make_cfg2_on_device(device, seed, n_streams, n_records, vsize, variant="A"):
    """Each stream: one v1 run of n_records Put records with sorted unique 16 B hex keys and
    random values, built directly in HBM (keys from splitmix64 on the host, values from the
    device RNG)."""
    from skv import gen

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    rec = 9 + 16 + vsize
    runs = []
    universe = 0 if variant == "A" else n_streams * n_records
    hdr = torch.tensor([1, 0, 0, 0, 16], dtype=torch.uint8, device=device)
    vl = torch.tensor(list(int(vsize).to_bytes(4, "big")), dtype=torch.uint8, device=device)
    for s in range(n_streams):
        ids = gen.unique_sorted_u64(seed + s, n_records, universe)
        keys = torch.from_numpy(np.ascontiguousarray(gen.hex16(ids))).to(device)
        run = torch.empty(1 + n_records * rec, dtype=torch.uint8, device=device)
        run[0] = 1
        body = run[1:].view(n_records, rec)
        body[:, 0:5] = hdr
        body[:, 5:21] = keys
        body[:, 21:25] = vl
        body[:, 25:] = torch.randint(0, 256, (n_records, vsize), dtype=torch.uint8, device=device, generator=g)
        runs.append(run)
    torch.cuda.synchronize(device)
    return runs


def cpu_baseline(sample_records, n_streams, vsize, repeats):
    """oracle/ (C restatement of read_run_stream + k_way::merge + build_runs, faithful shape,
    single thread) on a bounded sample: same shape, n_streams x sample_records records."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from skv import gen

    streams = gen.config2(seed=0xC0FFEE, n_streams=n_streams, n_records=sample_records, vsize=vsize)
    nbytes = gen.total_bytes(streams)
    pyoracle.compact(streams, MAX_RUN)  # warm-up
    ts = []
    for _ in range(repeats):
        t0 = time.perf_counter()
        pyoracle.compact(streams, MAX_RUN)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    return {
        "value": round(nbytes / t / GiB, 4),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{n_streams} streams x {sample_records} records x {9 + 16 + vsize} B = {nbytes / 2**20:.1f} MiB "
                  f"(config-2 shape, 1/{round(238821 / sample_records)} of the records), median of {repeats} after 1 warm-up",
        "seconds_per_run": round(t, 3),
    }


def rank_seed(rank):
    """Distinct synthetic inputs per rank: N independent compactions (BASELINE config 4)."""
    return 0x5EEDC0DE + 1000 * rank


def reduce_over_ranks(elapsed, in_bytes, dist, device):
    """(max elapsed over ranks, total input bytes over ranks): whole-job throughput is the
    units all ranks processed / the slowest rank's time. No data-path collective exists."""
    if dist is None:
        return elapsed, float(in_bytes)
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    b = torch.tensor([float(in_bytes)], dtype=torch.float64, device=device)
    dist.all_reduce(b, op=dist.ReduceOp.SUM)
    return float(t.item()), float(b.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--streams", type=int, default=64)
    ap.add_argument("--records", type=int, default=238821)
    ap.add_argument("--vsize", type=int, default=256)
    ap.add_argument("--variant", default="A")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-path", action="store_true", help="skip the PCIe-inclusive host-memory figure")
    ap.add_argument("--cpu-sample-records", type=int, default=238821 // 16)
    ap.add_argument("--cpu-repeats", type=int, default=3)
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="per-launch HBM bytes of each kernel measured with rocprofv3 --pmc (tools/traffic.py)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)

    from skv.api import Compactor

    seed = rank_seed(rank)
    runs = make_cfg2_on_device(device, seed, args.streams, args.records, args.vsize, args.variant)
    in_bytes = sum(r.numel() for r in runs)
    streams = [(s + 1, [(r.data_ptr(), r.numel())]) for s, r in enumerate(runs)]
    comp = Compactor(local_rank, profiling=True)

    out_bytes = 0
    n_out_runs = 0
    for _ in range(args.warmup):
        res = comp.compact_dev(streams, MAX_RUN, 0)
        out_bytes, n_out_runs = res.n_bytes, res.n_runs
        res.free()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(device)

    gather_ms, total_ms, phases, host_ms, sync_ms, call_ms = [], [], [], [], [], []
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tc = time.perf_counter()
        res = comp.compact_dev(streams, MAX_RUN, 0)
        call_ms.append((time.perf_counter() - tc) * 1e3)
        t = comp.timings()
        host_ms.append(t["host_total_ms"])
        sync_ms.append(t["host_sync_ms"])
        gather_ms.append(t["hot_ms"])
        total_ms.append(t["total_ms"])
        phases.append([t[k] for k in ("parse_ms", "check_ms", "merge_ms", "chain_ms", "gather_ms")])
        gread, gwrite = t["hot_read_bytes"], t["hot_write_bytes"]
        path = t["path"]
        out_bytes, n_out_runs = res.n_bytes, res.n_runs
        res.free()
    barrier()
    elapsed, total_in = reduce_over_ranks(time.perf_counter() - t0, in_bytes, dist, device)

    # PCIe-inclusive figure (not `value`): the host entry point skv_compact with the inputs in
    # pinned host memory and the output runs returned in pinned host memory.
    host_path = None
    if rank == 0 and world == 1 and not args.no_host_path:
        host_runs = [r.cpu().pin_memory() for r in runs]
        hstreams = [(s + 1, [(r.data_ptr(), r.numel())]) for s, r in enumerate(host_runs)]
        comp.compact_host_ptrs(hstreams, MAX_RUN, 0)  # warm-up (allocates the staging buffers)
        hts = []
        for _ in range(2):
            t1 = time.perf_counter()
            hb, _ = comp.compact_host_ptrs(hstreams, MAX_RUN, 0)
            hts.append(time.perf_counter() - t1)
        ht = min(hts)
        host_path = {"value": round(in_bytes / ht / GiB, 3), "unit": "GiB/s", "ms": round(ht * 1e3, 3),
                     "h2d_bytes": in_bytes, "d2h_bytes": hb,
                     "note": "skv_compact: pinned host inputs -> HBM -> compaction -> pinned host output, "
                             "best of 2 after 1 warm-up, serial copies (no overlap)"}
        del host_runs

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = total_in * args.steps / elapsed / GiB
        g_ms = float(np.mean(gather_ms))
        achieved = (gread + gwrite) / (g_ms * 1e-3) / 1e9
        traffic = None
        try:
            with open(args.traffic_json) as f:
                kt = json.load(f).get("kernels", {}).get("skv::" + HOT_KERNEL.get(path, "?"))
                traffic = kt["hbm_bytes"] if kt else None
        except (OSError, ValueError):
            traffic = None
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: splitmix64 sorted unique hex keys + device-RNG values, built in HBM",
            "config": {
                "workload": f"config 2{args.variant}: {args.streams}-way L0->L1 compaction, {args.streams} x 1 run x "
                            f"{args.records} records ({9 + 16 + args.vsize} B: 16 B keys / {args.vsize} B values), "
                            f"max run 4 MiB, one independent compaction per GPU",
                "streams": args.streams,
                "input_bytes_per_gpu": in_bytes,
                "output_bytes_per_gpu": out_bytes,
                "output_runs_per_gpu": n_out_runs,
                "parallelism": f"{world} independent compactions (one per GPU), no collective",
            },
            "device_ms_per_compaction": round(float(np.mean(total_ms)), 4),
            "host_ms": {"python_call": round(float(np.mean(call_ms)), 4),
                        "library": round(float(np.mean(host_ms)), 4),
                        "in_syncs": round(float(np.mean(sync_ms)), 4)},
            "phases_ms": dict(zip(("parse", "check", "merge", "chain", "gather"),
                                  [round(float(x), 4) for x in np.mean(np.array(phases), axis=0)])),
            "roofline": {
                "bound": "hbm",
                "kernel": HOT_KERNEL.get(path, "?"),
                "path": PATH_NAMES.get(path, "?"),
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": int(gread + gwrite),
                "avg_launch_ms": round(g_ms, 4),
                # whole compaction against the same peak: SURVEY §8d's (I + O) / t
                "pipeline_achieved": round((in_bytes + out_bytes) / (ms_per_step * 1e-3) / 1e9, 1),
                "pipeline_frac": round((in_bytes + out_bytes) / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            },
        }
        if host_path is not None:
            line["host_path"] = host_path
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.cpu_sample_records, args.streams, args.vsize, args.cpu_repeats)
        print(json.dumps(line), flush=True)
    comp.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
