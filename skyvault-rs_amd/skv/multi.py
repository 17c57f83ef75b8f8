"""Independent compactions across the GPUs of one node (BASELINE config 4).

The path shards with no exchange: each compaction (one table's buffer, one tree level, one WAL
flush; orchestrator_service.rs:119-170 schedules them independently) runs whole on one GPU.
`MultiCompactor` keeps one skv_ctx and one host thread per device; `submit` queues a compaction
to the device with the least queued input bytes (the jobs differ in size, so round-robin would
leave GPUs idle behind one large job) and returns a Future. The C call releases the GIL, so the
device threads run their compactions concurrently. There is no collective and no RCCL: results
come back to the caller's thread through the futures.
"""
from __future__ import annotations

import os
import queue
import threading
from concurrent.futures import Future
from typing import Callable, List, Optional, Sequence, Set


SYSFS_ROOT = "/sys"  # tests point this at a stub tree (the library's skv_host_plan takes the same root)


def numa_cpus(node: int) -> Set[int]:
    """CPUs of NUMA node `node` that this process may run on (sysfs cpulist; empty if unknown)."""
    try:
        with open(f"{SYSFS_ROOT}/devices/system/node/node{int(node)}/cpulist") as f:
            text = f.read().strip()
    except OSError:
        return set()
    cpus = set()
    for part in filter(None, text.split(",")):
        a, _, b = part.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    try:
        cpus &= os.sched_getaffinity(0)
    except (AttributeError, OSError):
        pass
    return cpus


class MultiCompactor:
    def __init__(self, devices: Sequence[int], factory: Optional[Callable[[int], object]] = None):
        """devices: HIP ordinals, one worker each (an ordinal may repeat: several ctxs on one GPU
        overlap one job's copies with another's kernels). factory(device) -> compactor; default
        skv.api.Compactor."""
        if factory is None:
            from .api import Compactor

            factory = Compactor
        self._lock = threading.Lock()
        self._workers: List[_Worker] = [_Worker(factory, d, self._lock) for d in devices]
        for w in self._workers:
            w.start()

    def submit(self, streams, max_run_size: int, flags: int = 0, with_info: bool = False,
               entry: str = "compact", then: Optional[Callable[[object, object], object]] = None) -> Future:
        """Queue one compaction. entry: the Compactor method that runs it -- "compact" (host run
        bytes, the default), "compact_dev" (device pointers: [(seq_no, [(ptr, len)])]) or
        "compact_host" (pinned host pointers). then(compactor, result), if given, runs on the
        worker's thread right after the call (e.g. to read the ctx's timings before its next
        call); the future holds its return value.

        A "compact_dev" result lives in the ctx's device output buffer, which the worker's next
        call on the same ctx overwrites (include/skv.h: valid until the next call on the ctx), so
        that entry requires `then`: read or copy the result there, before the worker moves on."""
        if entry not in ("compact", "compact_dev", "compact_host"):
            raise ValueError(f"unknown entry {entry!r}")
        if entry == "compact_dev" and then is None:
            raise ValueError('entry="compact_dev" needs then=: its DeviceResult is valid only until the '
                             "worker's next call on the same ctx")
        size = sum(len(r) if isinstance(r, (bytes, bytearray, memoryview)) else r[1]
                   for _, runs in streams for r in runs)
        with self._lock:
            w = min(self._workers, key=lambda x: x.queued_bytes)
            w.queued_bytes += size
        fut: Future = Future()
        w.q.put((streams, max_run_size, flags, with_info, entry, then, size, fut))
        return fut

    def map(self, jobs: Sequence[tuple]) -> List[object]:
        """jobs: [(streams, max_run_size, flags)] -> results in job order (raises the first error)."""
        futs = [self.submit(*j) for j in jobs]
        return [f.result() for f in futs]

    def close(self):
        for w in self._workers:
            w.q.put(None)
        for w in self._workers:
            w.join()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class _Worker(threading.Thread):
    def __init__(self, factory, device: int, lock: threading.Lock):
        super().__init__(daemon=True)
        self.lock = lock
        self.factory = factory
        self.device = device
        self.q: "queue.Queue" = queue.Queue()
        self.queued_bytes = 0
        self.error: Optional[BaseException] = None
        self.cpus: Set[int] = set()  # the NUMA-node CPUs this worker is bound to (empty: not bound)

    def run(self):
        try:
            comp = self.factory(self.device)  # the ctx is created and used on this thread only
        except BaseException as e:  # every later job fails with the ctx error
            comp, self.error = None, e
        # this device's host thread runs near its GPU: bound to the CPUs of the GPU's NUMA node (the
        # library allocates the ctx's pinned buffers there and runs its table passes on a pool bound
        # there too), so eight devices' host work does not cross the socket link
        info = getattr(comp, "host_info", None)
        if info is not None:
            try:
                cpus = numa_cpus(info()["numa_node"])
                if cpus:
                    os.sched_setaffinity(0, cpus)
                    self.cpus = cpus
            except (OSError, ValueError, KeyError):
                pass
        while True:
            item = self.q.get()
            if item is None:
                break
            streams, max_run_size, flags, with_info, entry, then, size, fut = item
            try:
                if comp is None:
                    raise self.error
                if entry == "compact":
                    res = comp.compact(streams, max_run_size, flags, with_info=with_info)
                else:
                    res = getattr(comp, entry)(streams, max_run_size, flags)
                fut.set_result(then(comp, res) if then is not None else res)
            except BaseException as e:
                fut.set_exception(e)
            finally:
                with self.lock:
                    self.queued_bytes -= size
        close = getattr(comp, "close", None)
        if close:
            close()
