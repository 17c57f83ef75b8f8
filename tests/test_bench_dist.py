"""N>1 path of bench.py on CPU (gloo, world size 2): each rank is an independent compaction
(distinct inputs), whole-job throughput = total input bytes of all ranks / slowest rank's time.
No data-path collective: the only cross-rank traffic is this reduction of two scalars."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    elapsed = 1.0 + rank  # rank 1 is the slow one
    in_bytes = (rank + 1) * 1000
    t, b = bench.reduce_over_ranks(elapsed, in_bytes, dist, torch.device("cpu"))
    q.put((rank, t, b, bench.rank_seed(rank)))
    dist.barrier()
    dist.destroy_process_group()


def test_reduce_over_ranks_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, t, b, _ in out:
        assert t == 2.0  # max over ranks
        assert b == 3000.0  # sum over ranks
    assert out[0][3] != out[1][3]  # independent compactions per rank


def test_single_rank_passthrough():
    sys.path.insert(0, ROOT)
    import bench

    assert bench.reduce_over_ranks(0.5, 123, None, torch.device("cpu")) == (0.5, 123.0)


def _compaction_worker(rank, world, port, q):
    """One rank of `bench.py --gpus 2` on CPU: its own compaction (bench.rank_seed(rank) inputs,
    config-2 shape, scaled down) run by the oracle through bench.timed_loop, the barrier on both
    sides, then bench.reduce_over_ranks — the same calls bench.main makes around the device."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "skyvault-rs_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import hashlib

    import bench
    import pyoracle
    from skv import gen

    streams = gen.config2(seed=bench.rank_seed(rank), n_streams=8, n_records=3000, vsize=64, variant="B")
    in_bytes = gen.total_bytes(streams)
    out = {}

    def step():
        out["runs"] = pyoracle.compact(streams, 64 * 1024, 0)

    elapsed = bench.timed_loop(step, 3, dist.barrier)
    t, b = bench.reduce_over_ranks(elapsed, in_bytes, dist, torch.device("cpu"))
    runs = out["runs"]
    digest = hashlib.sha256(b"".join(r.data for r in runs)).hexdigest()
    q.put((rank, elapsed, t, b, in_bytes, len(runs), digest, all(len(r.data) <= 64 * 1024 for r in runs)))
    dist.barrier()
    dist.destroy_process_group()


def test_each_rank_runs_its_own_compaction_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_compaction_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, e0, t0, b0, i0, n0, d0, ok0), (r1, e1, t1, b1, i1, n1, d1, ok1) = out
    assert t0 == t1 == max(e0, e1)  # every rank reports the slowest rank's time
    assert b0 == b1 == float(i0 + i1)  # whole-job bytes = all ranks' inputs
    assert d0 != d1 and n0 > 1 and n1 > 1 and ok0 and ok1  # independent compactions, split at max
