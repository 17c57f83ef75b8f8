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
