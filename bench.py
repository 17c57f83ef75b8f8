#!/usr/bin/env python3
"""Compaction throughput on MI355X — BASELINE.json's metric:
"compaction GiB/s of input run bytes merged (device-resident), 1/2/4/8 GPU".

Workload (BASELINE.json configs[1], SURVEY.md §8d config 2 variant A): a 64-way L0->L1
compaction of 64 streams x 1 run x 238,821 records (16 B hex keys, 256 B values, 281 B per
record, 67,108,702 B per run, 4.0 GiB total), max run size 4 MiB, no tombstones. One step
= one whole compaction (decode, merge, dedup, greedy split, stats, output bytes) with the
inputs already resident in HBM. At N GPUs every rank runs its own independent compaction
(distinct seeds; BASELINE config 4 at N=8): weak scaling, no collective on the data path.

Prints ONE JSON line on rank 0 with `roofline` (the dominant kernel: algorithmic bytes / its
HIP-event-timed duration on the library stream) and `cpu_baseline` (the C restatement in
oracle/, faithful shape, 1 core, on a bounded sample of the same workload).

--config selects the other BASELINE shapes for measurement records (never the default line):
  2B  config 2 with keys from a universe of |R| ids (~37 % superseded)
  3   256 streams of variable-length keys (8-128 B alnum) + 10 % Deletes, runs of --run-mib MiB
      (default 16: 1/16 of BASELINE's 256 MiB runs), built on the host, general path
  5   10^6 WAL runs x 83 records (32 B "{table}.{suffix}" keys, 8 B values), SKV_SPLIT_BY_TABLE,
      built in HBM; max run size 2^62 so every table keeps its one run (at the reference's 4 MiB
      every table of this size would be dropped by the exactly-one-run rule)
  L0  a table-buffer compaction as table_buffer_compaction.rs:31-100 builds it: 16 buffer runs
      (SeqNo 1..16) + ONE stream at SeqNo 0 concatenating 1,024 ascending L0 runs (4 MiB each,
      config 2's records), built in HBM
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
HOT_KERNEL = {1: "k_gather", 2: "k_gather", 3: "k_fx_tile"}  # config 5 (WAL stage): k_wal_gather
PATH_NAMES = {1: "general", 2: "fixed", 3: "fused"}
GiB = float(1 << 30)


def cpu_baseline(config, sample_records, n_streams, vsize, repeats, run_mib=16):
    """oracle/ (C restatement of read_run_stream + k_way::merge + build_runs, faithful shape,
    single thread) on a bounded sample of the same shape."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from skv import gen

    flags, max_run = 0, MAX_RUN
    if config in ("2A", "2B"):
        streams = gen.config2(seed=0xC0FFEE, n_streams=n_streams, n_records=sample_records, vsize=vsize,
                              variant=config[1])
        sample = (f"{n_streams} streams x {sample_records} records x {9 + 16 + vsize} B (config-{config} shape, "
                  f"1/{round(238821 / sample_records)} of the records)")
    elif config == "L0":
        streams = gen.config_l0(seed=0xC0FFEE, n_buffer=16, n_l0=1024, run_records=14925 // 16)
        sample = "16 buffer runs + one stream of 1,024 L0 runs, 932 records each (config-L0 shape, 1/16 of the records)"
    elif config in ("3", "3F"):
        # runs of run_mib / 16 MiB, at most 1 MiB (the bench's own runs are run_mib MiB: 16 for
        # config 3, 256 for 3F)
        sample_bytes = (min(run_mib, 16) << 20) // 16
        streams = gen.config3(seed=0xC0FFEE, n_streams=n_streams, run_bytes=sample_bytes)
        sample = (f"{n_streams} streams x {sample_bytes / 2**20:.2f} MiB runs (config-{config} shape, "
                  f"1/{round((run_mib << 20) / sample_bytes)} of the bench's {run_mib} MiB runs)")
    else:
        from skv import _abi
        from skv.devgen import make_cfg5_on_device

        n5 = 20000
        host = make_cfg5_on_device(torch.device("cuda", torch.cuda.current_device()), 0xC0FFEE, n5).cpu().numpy()
        rl = host.shape[1]
        table5 = _abi.stream_table(np.arange(1, n5 + 1), host.ctypes.data + rl * np.arange(n5, dtype=np.uint64),
                                   np.full(n5, rl))
        flags, max_run = 2, 1 << 62
        sample = f"{n5:,} WAL runs x 83 records (config-5 shape, 1/50 of the streams)"
        streams = None
    nbytes = gen.total_bytes(streams) if streams is not None else host.size

    def run_once():
        if streams is not None:
            pyoracle.compact(streams, max_run, flags)
        else:
            pyoracle.compact_np(table5, max_run, flags)

    run_once()  # warm-up
    ts = []
    for _ in range(repeats):
        t0 = time.perf_counter()
        run_once()
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    out = {
        "value": round(nbytes / t / GiB, 4),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{sample} = {nbytes / 2**20:.1f} MiB, median of {repeats} after 1 warm-up",
        "seconds_per_run": round(t, 3),
    }
    out.update(host_cpu())
    if config == "2A":
        out["config4_8_compactions"] = cpu_baseline_config4(sample_records, n_streams, vsize, repeats)
    return out


def host_cpu():
    """The box's host CPU as cpu_baseline reports it: logical CPUs and the model name."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "cpu_model": model}


def cpu_baseline_config4(sample_records, n_streams, vsize, repeats):
    """BASELINE config 4's CPU leg: 8 independent compactions of the config-2A
    shape (distinct seeds, each a bounded sample) on min(8, nproc) threads — the oracle releases
    the GIL inside its C call, so the threads run in parallel."""
    from concurrent.futures import ThreadPoolExecutor

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from skv import _abi, gen

    jobs = []
    for j in range(8):
        streams = gen.config2(seed=0xC0FFEE + 1000 * j, n_streams=n_streams, n_records=sample_records, vsize=vsize)
        bufs = [np.frombuffer(r[1][0], dtype=np.uint8) for r in streams]
        jobs.append((bufs, _abi.stream_table(np.arange(1, n_streams + 1), [b.ctypes.data for b in bufs],
                                             [b.size for b in bufs])))
    nbytes = sum(b.size for bufs, _ in jobs for b in bufs)
    threads = min(8, os.cpu_count() or 1)

    def one(job):
        pyoracle.compact_np(job[1], MAX_RUN, 0)

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(one, jobs))  # warm-up
        ts = []
        for _ in range(repeats):
            t0 = time.perf_counter()
            list(ex.map(one, jobs))
            ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    return {"value": round(nbytes / t / GiB, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"8 independent config-2A compactions (distinct seeds), each {n_streams} streams x "
                      f"{sample_records} records = {nbytes / 8 / 2**20:.1f} MiB, on {threads} threads, "
                      f"median of {repeats} after 1 warm-up"}


def check_invariants(res, config, max_run, in_records):
    """Size-independent properties of one full-size result (the bench's own input; bit-exact parity
    at these sizes is tests/test_gpu_fullsize.py): byte accounting, run sizes under the greedy
    split, record counts. Raises on a violation."""
    d = res.descs
    assert res.n_runs == len(d)
    assert sum(x[1] for x in d) == res.n_bytes, "run lengths != output bytes"
    off = 0
    for x in d:  # contiguous runs, each within max (or a single record)
        assert x[0] == off, "runs not contiguous"
        assert x[1] <= max_run or x[2] + x[3] == 1, "run above max with more than one record"
        off += x[1]
    assert sum(x[2] + x[3] for x in d) == res.out_records
    if config == "2A":  # no key repeats across streams (2^64 key space): every record survives
        assert res.out_records == in_records
        assert res.n_bytes == res.in_bytes - 64 + res.n_runs
    return {"checked": True, "runs": len(d), "out_records": res.out_records}


def config4_one_gpu(device, dev_idx, runs0, n_streams, n_records, vsize, max_run, reps=3):
    """BASELINE config 4's workload on ONE GPU (never `value`): 8 independent config-2A compactions
    (the rank seeds 0..7 of the 8-GPU run) submitted together to skv.multi.MultiCompactor, one ctx
    and worker thread each, all on this device -- eight calls in flight on eight HIP streams. Wall
    time per batch of 8, best of `reps` after one warm-up batch."""
    from skv.devgen import make_cfg2_on_device
    from skv.multi import MultiCompactor

    inputs = [runs0] + [make_cfg2_on_device(device, rank_seed(j), n_streams, n_records, vsize, "A") for j in range(1, 8)]
    tables = [[(s + 1, [(r.data_ptr(), r.numel())]) for s, r in enumerate(runs)] for runs in inputs]
    in_bytes = sum(r.numel() for runs in inputs for r in runs)

    def done(comp, res):  # on the worker thread: the path taken, then give the output back
        p = comp.timings()["path"]
        res.free()
        return p

    walls, paths = [], set()
    with MultiCompactor([dev_idx] * 8) as mc:
        for rep in range(reps + 1):
            torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            futs = [mc.submit(t, max_run, 0, entry="compact_dev", then=done) for t in tables]
            paths.update(f.result() for f in futs)
            torch.cuda.synchronize(device)
            if rep:
                walls.append(time.perf_counter() - t0)
    del inputs, tables
    torch.cuda.empty_cache()
    w = min(walls)
    return {"value": round(in_bytes / w / GiB, 3), "unit": "GiB/s", "ms_per_batch": round(w * 1e3, 3),
            "ms_per_compaction": round(w * 1e3 / 8, 4), "input_bytes": in_bytes,
            "paths": sorted(PATH_NAMES.get(p, "?") for p in paths),
            "note": "config 4 on one GPU: 8 config-2A compactions (rank seeds 0..7) submitted at once to "
                    "MultiCompactor, 8 ctxs + worker threads on this device; wall per batch of 8, best of "
                    f"{reps} after 1 warm-up batch (the 8-GPU figure is the driver's --gpus 8 run)"}


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


def split_extra(devices, hstreams, max_run, flags, in_bytes, reps=2):
    """skv_compact_split over one ctx per entry of `devices` (pinned host inputs, pinned host output):
    GiB/s of input bytes, best of `reps` after 1 warm-up, beside the same call through skv_compact
    on the first device alone. Never the bench's outcome: an error is recorded, not raised."""
    from skv.api import Compactor, compact_split

    try:
        cs = [Compactor(d) for d in devices]
        try:
            compact_split(cs, hstreams, max_run, flags, keep=True).free()
            best = None
            for _ in range(reps):
                t1 = time.perf_counter()
                r = compact_split(cs, hstreams, max_run, flags, keep=True)
                dt = time.perf_counter() - t1
                best = dt if best is None else min(best, dt)
                out_b = r.n_bytes
                r.free()
            parts = int(cs[0].timings()["host_parts"])
            cs[0].compact_host_ptrs(hstreams, max_run, flags)
            one = None
            for _ in range(reps):
                t1 = time.perf_counter()
                cs[0].compact_host_ptrs(hstreams, max_run, flags)
                dt = time.perf_counter() - t1
                one = dt if one is None else min(one, dt)
        finally:
            for c in cs:
                c.close()
        return {"value": round(in_bytes / best / GiB, 3), "unit": "GiB/s", "ms": round(best * 1e3, 3),
                "ctxs": len(devices), "devices": sorted(set(devices)), "parts": parts, "d2h_bytes": out_b,
                "one_ctx_value": round(in_bytes / one / GiB, 3),
                "note": f"skv_compact_split over {len(devices)} ctxs (key-range parts dealt round-robin; each "
                        "part's H2D and kernels on its ctx, its D2H once the output size of every earlier part "
                        f"is known), pinned host in/out, best of {reps} after 1 warm-up; one_ctx_value: "
                        "skv_compact on the first device alone"}
    except Exception as e:  # a figure for the record, never the bench's outcome
        return {"value": None, "error": f"{type(e).__name__}: {e}"}


def timed_loop(step, steps, barrier):
    """The bench contract's timed region: barrier (+ device sync) on both sides of exactly `steps`
    calls of step(); returns this rank's elapsed seconds (reduce_over_ranks takes the max)."""
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    barrier()
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--streams", type=int, default=64)
    ap.add_argument("--records", type=int, default=238821)
    ap.add_argument("--vsize", type=int, default=256)
    ap.add_argument("--variant", default="A", help="config 2 variant (same as --config 2A / 2B)")
    ap.add_argument("--config", default=None, choices=["2A", "2B", "3", "3F", "5", "L0"])
    ap.add_argument("--run-mib", type=int, default=16, help="config 3 run size")
    ap.add_argument("--wal-runs", type=int, default=1_000_000, help="config 5 stream count")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true",
                    help="diagnostic library builds only (output invalid by design): skip the invariants")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the extra figures: PCIe-inclusive host memory, two ctxs in flight")
    ap.add_argument("--cpu-sample-records", type=int, default=238821 // 16)
    ap.add_argument("--cpu-repeats", type=int, default=5)
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="per-launch HBM bytes of each kernel measured with rocprofv3 --pmc (tools/traffic.py)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        # gloo over the host: the path shards with no data-path exchange (north_star: no RCCL), so
        # the only cross-rank traffic is the start/stop barrier and two scalars
        dist.init_process_group("gloo")
    # SKV_BENCH_SHARE_DEVICE=1: every rank on device 0 -- a rehearsal of the N-rank path on a
    # one-GPU box (the line then says so; its value is not a scaling figure)
    shared = os.environ.get("SKV_BENCH_SHARE_DEVICE") == "1"
    dev_idx = 0 if shared else local_rank
    torch.cuda.set_device(dev_idx)
    device = torch.device("cuda", dev_idx)

    from skv.api import Compactor
    from skv.devgen import (make_cfg2_on_device, make_cfg3_full_on_device, make_cfg3_on_device, make_cfg5_on_device,
                            make_l0_on_device)

    seed = rank_seed(rank)
    config = args.config or "2" + args.variant
    run_mib_used = (256 if args.run_mib == 16 else args.run_mib) if config == "3F" else args.run_mib
    flags, max_run = 0, MAX_RUN
    if config in ("2A", "2B"):
        runs = make_cfg2_on_device(device, seed, args.streams, args.records, args.vsize, config[1])
        workload = (f"config {config}: {args.streams}-way L0->L1 compaction, {args.streams} x 1 run x {args.records} "
                    f"records ({9 + 16 + args.vsize} B: 16 B keys / {args.vsize} B values), max run 4 MiB, "
                    f"one independent compaction per GPU")
        data = "synthetic: splitmix64 sorted unique hex keys + device-RNG values, built in HBM"
        n_streams = args.streams
    elif config == "3F":
        n_streams = 256 if args.streams == 64 else args.streams
        run_mib = 256 if args.run_mib == 16 else args.run_mib
        runs = make_cfg3_full_on_device(device, seed, n_streams, run_mib)
        workload = (f"config 3: {n_streams}-way compaction, {n_streams} x 1 run of ~{run_mib} MiB, variable-length "
                    f"keys 8-128 B + 10 % Deletes, 256 B values, max run 4 MiB")
        data = "synthetic: sorted unique ids rendered as order-preserving alnum keys + alnum tails, built in HBM"
    elif config == "L0":
        bruns, lruns = make_l0_on_device(device, seed)
        runs = bruns + lruns
        n_streams = len(bruns) + 1
        workload = (f"table-buffer compaction with L0: {len(bruns)} buffer runs (SeqNo 1..{len(bruns)}) + one stream "
                    f"at SeqNo 0 concatenating {len(lruns)} ascending L0 runs of 14,925 records (281 B: 16 B keys / "
                    f"256 B values, 4 MiB runs), max run 4 MiB")
        data = "synthetic: splitmix64 ids from one universe (buffer records supersede some L0 records), built in HBM"
    elif config == "3":
        n_streams = 256 if args.streams == 64 else args.streams
        runs = make_cfg3_on_device(device, seed, n_streams, args.run_mib)
        workload = (f"config 3 (scaled): {n_streams}-way compaction, {n_streams} x 1 run of ~{args.run_mib} MiB, "
                    f"variable-length keys 8-128 B + 10 % Deletes, 256 B values, max run 4 MiB")
        data = "synthetic: gen.config3 (splitmix64 ids, alnum keys sorted bytewise), host-built, copied to HBM"
    else:
        n_streams = args.wal_runs
        buf = make_cfg5_on_device(device, seed, n_streams)
        runs = [buf]
        flags, max_run = 2, 1 << 62
        workload = (f"config 5: WAL -> table-buffer flush, {n_streams} WAL runs x 83 records (32 B keys / 8 B values, "
                    f"4,068 B runs), SKV_SPLIT_BY_TABLE over 64 tables, one run per table")
        data = "synthetic: device-RNG table ids and suffixes, runs sorted in HBM"
    if config == "5":
        rl = buf.shape[1]
        base = buf.data_ptr()
        in_bytes = buf.numel()
        streams = [(s + 1, [(base + s * rl, rl)]) for s in range(n_streams)]
    elif config == "L0":
        in_bytes = sum(r.numel() for r in runs)
        streams = [(b + 1, [(r.data_ptr(), r.numel())]) for b, r in enumerate(bruns)]
        streams.append((0, [(r.data_ptr(), r.numel()) for r in lruns]))
    else:
        in_bytes = sum(r.numel() for r in runs)
        streams = [(s + 1, [(r.data_ptr(), r.numel())]) for s, r in enumerate(runs)]
    comp = Compactor(dev_idx, profiling=True)
    # the skv_stream[] table, built once like a caller's Vec (at 10^6 streams building it in Python
    # costs more than the compaction)
    from skv._abi import StreamArgs

    table = StreamArgs(streams, device=True)

    out_bytes = 0
    n_out_runs = 0
    for _ in range(args.warmup):
        res = comp.compact_dev(table, max_run, flags)
        out_bytes, n_out_runs = res.n_bytes, res.n_runs
        res.free()

    def barrier():
        torch.cuda.synchronize(device)
        if dist is not None:
            dist.barrier()

    gather_ms, total_ms, phases, host_ms, sync_ms, call_ms = [], [], [], [], [], []
    last = {}

    def step():
        tc = time.perf_counter()
        res = comp.compact_dev(table, max_run, flags)
        call_ms.append((time.perf_counter() - tc) * 1e3)
        t = comp.timings()
        host_ms.append(t["host_total_ms"])
        sync_ms.append(t["host_sync_ms"])
        gather_ms.append(t["hot_ms"])
        total_ms.append(t["total_ms"])
        phases.append([t[k] for k in ("parse_ms", "check_ms", "merge_ms", "chain_ms", "gather_ms")])
        last.update(t=t, out=(res.n_bytes, res.n_runs))
        res.free()

    elapsed_rank = timed_loop(step, args.steps, barrier)
    t = last["t"]
    gread, gwrite, path = t["hot_read_bytes"], t["hot_write_bytes"], t["path"]
    out_bytes, n_out_runs = last["out"]
    # invariants of the measured call's output (outside the timed region)
    res = comp.compact_dev(table, max_run, flags)
    if args.no_check:
        invariants = {"checked": False, "note": "--no-check (diagnostic build)"}
    else:
        invariants = check_invariants(res, config, max_run, res.in_records) if config != "5" else {
            "checked": True, "runs": res.n_runs, "out_records": res.out_records}
    res.free()
    elapsed, total_in = reduce_over_ranks(elapsed_rank, in_bytes, dist, torch.device("cpu"))

    # Not `value`: the same compaction issued from 2 host threads on 2 ctxs (2 HIP streams) of this
    # GPU, 2 calls in flight -- one call's splitter phase and host gaps beside the other's tile phase
    # (tools/overlap_probe.py). ms per compaction = wall / calls.
    concurrent = None
    if rank == 0 and world == 1 and config in ("2A", "2B") and not args.no_host_path:
        import threading

        comps = [Compactor(dev_idx), Compactor(dev_idx)]  # (no per-phase event timing on these)
        for c in comps:
            c.compact_dev(table, max_run, flags).free()
        n_each = max(10, args.steps)

        def worker(c):
            for _ in range(n_each):
                c.compact_dev(table, max_run, flags).free()

        th = [threading.Thread(target=worker, args=(c,)) for c in comps]
        torch.cuda.synchronize(device)
        t1 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        torch.cuda.synchronize(device)
        dt = time.perf_counter() - t1
        concurrent = {"value": round(in_bytes * 2 * n_each / dt / GiB, 3), "unit": "GiB/s",
                      "ms_per_compaction": round(dt / (2 * n_each) * 1e3, 4), "calls": 2 * n_each,
                      "note": "2 ctxs x %d skv_compact_dev calls from 2 host threads, same inputs; wall / calls"
                              % n_each}
        for c in comps:
            c.close()

    config4 = None

    # PCIe-inclusive figure (not `value`): the host entry point skv_compact with the inputs in
    # pinned host memory and the output runs returned in pinned host memory.
    host_path = None
    # 3F at its full 256 MiB runs would pin 64 GB of host memory: its host figure is taken on runs of
    # at most 64 MiB (--run-mib 64: 256 x 64 MiB = 16 GiB pinned)
    if rank == 0 and world == 1 and not args.no_host_path and not (config == "3F" and run_mib_used > 64):
        if config == "5":  # one pinned buffer of 10^6 WAL runs; the stream table built once
            host_runs = [buf.cpu().pin_memory()]
            hb0 = host_runs[0].data_ptr()
            hstreams = StreamArgs([(s + 1, [(hb0 + s * rl, rl)]) for s in range(n_streams)], device=True)
        elif config == "L0":
            host_runs = [r.cpu().pin_memory() for r in runs]
            nb_ = len(bruns)
            hstreams = [(b + 1, [(r.data_ptr(), r.numel())]) for b, r in enumerate(host_runs[:nb_])]
            hstreams.append((0, [(r.data_ptr(), r.numel()) for r in host_runs[nb_:]]))
        else:
            host_runs = [r.cpu().pin_memory() for r in runs]
            hstreams = [(s + 1, [(r.data_ptr(), r.numel())]) for s, r in enumerate(host_runs)]
        comp.compact_host_ptrs(hstreams, max_run, flags)  # warm-up (allocates the staging buffers)
        hts = []
        for _ in range(2):
            t1 = time.perf_counter()
            hb, _ = comp.compact_host_ptrs(hstreams, max_run, flags)
            hts.append(time.perf_counter() - t1)
        ht = min(hts)
        parts = int(comp.timings()["host_parts"])
        # the drop-in entry point's own output, checked like the device line's (bit-exact parity at
        # this size: tests/test_gpu_fullsize.py::test_config*_host_entry_full_size)
        hr = comp.compact_host(hstreams, max_run, flags)
        host_inv = check_invariants(hr, config, max_run, hr.in_records)
        host_inv["parts"] = int(comp.timings()["host_parts"])
        hr.free()
        host_path = {"value": round(in_bytes / ht / GiB, 3), "unit": "GiB/s", "ms": round(ht * 1e3, 3),
                     "h2d_bytes": in_bytes, "d2h_bytes": hb, "parts": parts, "invariants": host_inv,
                     "note": "skv_compact: pinned host inputs -> HBM -> compaction -> pinned host output, "
                             "best of 2 after 1 warm-up, " + (
                                 f"{parts} key-range parts with H2D, kernels and D2H overlapped" if parts
                                 else "serial copies (no overlap)")}
        # two ctxs (two HIP streams) on the same GPU, each compacting from its own host thread:
        # one job's D2H overlaps the next job's H2D on the separate copy engines (skv.h threading
        # contract: different ctxs run concurrently)
        import threading

        comp2 = Compactor(dev_idx)
        comp2.compact_host_ptrs(hstreams, max_run, flags)
        n_jobs = 3

        def worker(c):
            for _ in range(n_jobs):
                c.compact_host_ptrs(hstreams, max_run, flags)

        th = [threading.Thread(target=worker, args=(c,)) for c in (comp, comp2)]
        t1 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        tp = time.perf_counter() - t1
        comp2.close()
        host_path["pipelined_2ctx"] = {
            "value": round(2 * n_jobs * in_bytes / tp / GiB, 3), "unit": "GiB/s",
            "note": f"2 ctxs x {n_jobs} skv_compact calls from 2 host threads, same pinned inputs"}
        if config in ("2A", "2B", "L0", "3"):
            # skv_compact_split: the same call as key-range parts over 4 ctxs. Here all
            # four share this GPU's PCIe link, so the figure is the split's overhead against the
            # pipelined single-ctx call, not its scaling (G GPUs move their parts over G links; the
            # N-GPU runs report split_ngpu)
            host_path["split_4ctx_1gpu"] = split_extra([dev_idx] * 4, hstreams, max_run, flags, in_bytes)
        del host_runs
        # the ceiling of this figure: the box's PCIe with both directions busy at once (1 GiB H2D on
        # one stream while 1 GiB D2H runs on another, pinned buffers); a host call moves its input
        # bytes in and about as many output bytes out, so value <= bidir / 2
        try:
            nb = 1 << 30
            dbuf_a = torch.empty(nb, dtype=torch.uint8, device=device)
            dbuf_b = torch.empty(nb, dtype=torch.uint8, device=device)
            h_a = torch.empty(nb, dtype=torch.uint8).pin_memory()
            h_b = torch.empty(nb, dtype=torch.uint8).pin_memory()
            s_in, s_out = torch.cuda.Stream(device), torch.cuda.Stream(device)
            best = None
            for _ in range(3):
                torch.cuda.synchronize(device)
                t1 = time.perf_counter()
                with torch.cuda.stream(s_in):
                    dbuf_a.copy_(h_a, non_blocking=True)
                with torch.cuda.stream(s_out):
                    h_b.copy_(dbuf_b, non_blocking=True)
                torch.cuda.synchronize(device)
                dt = time.perf_counter() - t1
                best = dt if best is None else min(best, dt)
            bidir = 2 * nb / best / 1e9
            host_path["pcie_bidir_GBps"] = round(bidir, 1)
            host_path["frac_of_pcie"] = round((in_bytes + hb) / ht / 1e9 / bidir, 3)
            del dbuf_a, dbuf_b, h_a, h_b
        except Exception as e:  # a figure for the record, never the bench's outcome
            host_path["pcie_bidir_GBps"] = f"unmeasured: {e}"

    # config 4 on this GPU after the host path: the host path measured after config 4's eight ctxs
    # and 34 GB of inputs had come and gone ran at 25.5 instead of 42 GiB/s (profiles/r05/h2a_order.txt)
    if (rank == 0 and world == 1 and config == "2A" and not args.no_host_path
            and os.environ.get("SKV_BENCH_CONFIG4", "1") != "0"):
        config4 = config4_one_gpu(device, dev_idx, runs, args.streams, args.records, args.vsize, max_run)

    # SURVEY §8(e) on N GPUs: rank 0's own input as ONE compaction split over all N GPUs of the node,
    # after the timed region (the other ranks' timed work is over; skv_compact_split drives every
    # device from this process, one host thread per shard). Not `value`, not part of the timing.
    split_ngpu = None
    # (SKV_BENCH_SHARE_DEVICE=1 rehearsals: N ctxs of device 0)
    if (rank == 0 and world > 1 and config in ("2A", "2B") and not args.no_host_path
            and os.environ.get("SKV_BENCH_SPLIT", "1") != "0"):
        host_runs = [r.cpu().pin_memory() for r in runs]
        hs = [(s + 1, [(r.data_ptr(), r.numel())]) for s, r in enumerate(host_runs)]
        split_ngpu = split_extra([0] * world if shared else list(range(world)), hs, max_run, flags, in_bytes)
        del host_runs

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = total_in * args.steps / elapsed / GiB
        g_ms = float(np.mean(gather_ms))
        whole_call = g_ms <= 0
        if whole_call:  # the exact WAL stage reports no single dominant launch: the whole device time
            g_ms = float(np.mean(total_ms))
        achieved = (gread + gwrite) / (g_ms * 1e-3) / 1e9
        hot_kernel = ("k_wal_fused" if t["wal_stage"] == 1 else "k_wal_gather") if config == "5" else HOT_KERNEL.get(path, "?")
        if whole_call:  # not a kernel roofline: say so
            hot_kernel = "call"
        # PMC counters of THIS config's dominant kernel (tools/traffic.py keys them by config and
        # kernel); none recorded -> null with the reason, never another config's counters
        traffic, traffic_note, traffic_rw = None, None, None
        call_traffic = None
        try:
            with open(args.traffic_json) as f:
                cfgs = json.load(f).get("configs", {})
            kt = cfgs.get(config, {}).get("kernels", {}).get("skv::" + hot_kernel)
            ct = cfgs.get(config, {}).get("call")
            if ct and not (config == "3F" and run_mib_used != 256):
                # every skv kernel's corrected PMC bytes over one whole call, against the call's I + O
                call_traffic = {"hbm_bytes": ct["hbm_bytes"], "read_bytes": ct["read_bytes"],
                                "write_bytes": ct["write_bytes"], "launches": ct["launches"],
                                "ratio_to_io": round(ct["hbm_bytes"] / max(1, in_bytes + out_bytes), 3),
                                "source": os.path.relpath(args.traffic_json, ROOT) + f" [configs][{config}][call]"}
            if config == "3F" and run_mib_used != 256:  # the recorded 3F pass is at 256 MiB runs
                kt, traffic_note = None, f"no --pmc pass recorded for config 3F at {run_mib_used} MiB runs"
            if kt:
                traffic = kt["hbm_bytes"]
                traffic_rw = {"read_bytes": kt["read_bytes"], "write_bytes": kt["write_bytes"],
                              "ratio_to_algorithmic": round(kt["hbm_bytes"] / max(1, gread + gwrite), 3),
                              "source": os.path.relpath(args.traffic_json, ROOT) + f" [configs][{config}]"}
            elif traffic_note is None:
                traffic_note = f"no --pmc pass recorded for config {config} / {hot_kernel} in {args.traffic_json}"
        except (OSError, ValueError) as e:
            traffic_note = f"traffic file unreadable: {e}"
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
            "data": data,
            "config": {
                "workload": workload,
                "streams": n_streams,
                "input_bytes_per_gpu": in_bytes,
                "output_bytes_per_gpu": out_bytes,
                "output_runs_per_gpu": n_out_runs,
                "parallelism": f"{world} independent compactions (one per GPU), no collective"
                               + (f" -- REHEARSAL: all {world} ranks share device 0" if shared else ""),
            },
            "device_ms_per_compaction": round(float(np.mean(total_ms)), 4),
            "host_ms": {"python_call": round(float(np.mean(call_ms)), 4),
                        "library": round(float(np.mean(host_ms)), 4),
                        "in_syncs": round(float(np.mean(sync_ms)), 4)},
            "phases_ms": dict(zip(("parse", "check", "merge", "chain", "gather"),
                                  [round(float(x), 4) for x in np.mean(np.array(phases), axis=0)])),
            "record_sort": bool(t["sorted"]),
            "roofline": {
                "bound": "hbm",
                "kernel": hot_kernel,
                "path": PATH_NAMES.get(path, "?"),
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_detail": traffic_rw if traffic is not None else traffic_note,
                "algorithmic_bytes_per_launch": int(gread + gwrite),
                "avg_launch_ms": round(g_ms, 4),
                # whole compaction against the same peak: SURVEY §8d's (I + O) / t
                "pipeline_achieved": round((in_bytes + out_bytes) / (ms_per_step * 1e-3) / 1e9, 1),
                "pipeline_frac": round((in_bytes + out_bytes) / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            },
            "call_traffic": call_traffic,
        }
        line["invariants"] = invariants
        if host_path is not None:
            line["host_path"] = host_path
        if split_ngpu is not None:
            line["split_ngpu"] = split_ngpu
        if concurrent is not None:
            line["concurrent_2ctx"] = concurrent
        if config4 is not None:
            line["config4_1gpu"] = config4
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(config, args.cpu_sample_records, n_streams if config != "5" else 0,
                                            args.vsize, args.cpu_repeats, run_mib_used)
        print(json.dumps(line), flush=True)
    comp.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
