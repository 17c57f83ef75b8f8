"""Multi-device placement on CPU (orchestrator_service.rs:119-170
places independent jobs one per GPU): a stubbed 8-GPU node, two NUMA nodes of four GPUs, as a stub
sysfs tree. No HIP device is touched -- the library's placement plans are pure functions
(skv_host_plan, skv_split_deal in include/skv.h) and MultiCompactor takes a stub compactor factory.

  - skv_host_plan: GPU j's NUMA node from its PCI device's numa_node, the node's CPUs its host pool is
    bound to, and the pool size (SKV_HOST_THREADS capped at CPUs / GPUs);
  - MultiCompactor([0..7]): job j runs on the worker of device j (one ctx per device, least queued
    bytes), all eight at once, each worker thread bound to the CPUs of its GPU's node;
  - skv_split_deal: part p of skv_compact_split on ctxs[p % G] (GPU p % G when ctx g is on GPU g),
    and the H2D order of ctxs that share a device.
"""
import os
import threading

import pytest

from skv import api, multi
from skv.multi import MultiCompactor

N_GPUS = 8
NODE_CPUS = {0: "0-3", 1: "4-7"}  # this container's 8 CPUs as two sockets of four


def _bus(j):
    return f"0000:{0x11 + 0x10 * j:02X}:00.0"  # upper case, as hipDeviceGetPCIBusId may report it


@pytest.fixture
def sysfs(tmp_path, monkeypatch):
    root = tmp_path / "sys"
    for j in range(N_GPUS):
        d = root / "bus" / "pci" / "devices" / _bus(j).lower()
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{j // 4}\n")
    for node, cpus in NODE_CPUS.items():
        d = root / "devices" / "system" / "node" / f"node{node}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpus + "\n")
    monkeypatch.setattr(multi, "SYSFS_ROOT", str(root))
    return str(root)


def _node_cpus(node):
    a, b = map(int, NODE_CPUS[node].split("-"))
    return set(range(a, b + 1))


def test_host_plan_per_gpu(sysfs):
    for j in range(N_GPUS):
        p = api.host_plan(_bus(j), N_GPUS, 256, sysfs)
        assert p["numa_node"] == j // 4
        assert set(p["cpus"]) == _node_cpus(j // 4)
        assert p["pool_threads"] == 8  # min(SKV_HOST_THREADS default 8, 256 CPUs / 8 GPUs)
    # a small host: the pool shrinks to CPUs / GPUs; an unknown device: no node, no binding
    assert api.host_plan(_bus(0), N_GPUS, 16, sysfs)["pool_threads"] == 2
    q = api.host_plan("0000:ff:00.0", N_GPUS, 256, sysfs)
    assert q["numa_node"] == -1 and q["cpus"] == []


class _StubDev:
    """A compactor stub for device d: host_info is the library's plan for GPU d (what
    skv_ctx_host_info reports for a live ctx); compact_dev records where it ran."""

    def __init__(self, device, sysfs, gate):
        self.device = device
        self.sysfs = sysfs
        self.gate = gate

    def host_info(self):
        p = api.host_plan(_bus(self.device), N_GPUS, 256, self.sysfs)
        return {"numa_node": p["numa_node"], "host_threads": p["pool_threads"]}

    def compact_dev(self, streams, max_run_size, flags):
        self.gate.wait(timeout=30)  # every job in flight at once: one worker thread per device
        return {"device": self.device, "thread": threading.get_ident(), "cpus": os.sched_getaffinity(0),
                "job": streams[0][0]}


@pytest.mark.skipif(not hasattr(os, "sched_setaffinity"), reason="no CPU affinity on this platform")
@pytest.mark.skipif(not _node_cpus(0) | _node_cpus(1) <= os.sched_getaffinity(0), reason="needs CPUs 0-7")
def test_eight_jobs_one_per_device_bound_to_its_node(sysfs):
    gate = threading.Barrier(N_GPUS)
    made = {}

    def factory(d):
        made[d] = _StubDev(d, sysfs, gate)
        return made[d]

    # eight equal jobs (config 4: one table compaction per GPU); device pointers are never read
    jobs = [[(j + 1, [(0x1000 * (j + 1), 64 << 20)])] for j in range(N_GPUS)]
    with MultiCompactor(list(range(N_GPUS)), factory) as mc:
        futs = [mc.submit(j, 4 << 20, 0, entry="compact_dev", then=lambda comp, res: res) for j in jobs]
        out = [f.result(timeout=60) for f in futs]
        bound = {w.device: w.cpus for w in mc._workers}
    assert sorted(made) == list(range(N_GPUS))
    for j, r in enumerate(out):
        assert r["job"] == j + 1 and r["device"] == j  # job j on device j
        assert r["cpus"] == _node_cpus(j // 4)  # its worker thread runs on its GPU's node
        assert bound[j] == _node_cpus(j // 4)
    assert len({r["thread"] for r in out}) == N_GPUS


def test_compact_dev_needs_then(sysfs):
    """a compact_dev result lives in the ctx's output buffer until the worker's next call"""
    with MultiCompactor([0], lambda d: _StubDev(d, sysfs, threading.Barrier(1))) as mc:
        with pytest.raises(ValueError):
            mc.submit([(1, [(0x1000, 64)])], 4 << 20, 0, entry="compact_dev")


def test_split_deal_one_ctx_per_gpu():
    ctx_of, after = api.split_deal(list(range(N_GPUS)), 3 * N_GPUS)
    assert ctx_of == [p % N_GPUS for p in range(3 * N_GPUS)]  # part p on GPU p % 8
    assert after == [-1] * (3 * N_GPUS)  # no two ctxs share a link: no H2D ordering


def test_split_deal_ctxs_sharing_devices():
    """four ctxs on two GPUs (0, 0, 1, 1): a part waits for the H2D of the latest earlier part of the
    OTHER ctx on its GPU, so each link takes its inputs in part order"""
    ctx_of, after = api.split_deal([0, 0, 1, 1], 10)
    assert ctx_of == [0, 1, 2, 3, 0, 1, 2, 3, 0, 1]
    assert after == [-1, 0, -1, 2, 1, 4, 3, 6, 5, 8]
    with pytest.raises(Exception):
        api.split_deal([], 4)
