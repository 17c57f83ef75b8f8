"""Host-side binding of libskv.so (include/skv.h) — the MI355X compaction path.

`Compactor` owns one skv_ctx (one GPU). Its `compact()` is the drop-in for the
read_run_stream -> k_way::merge -> [filter] -> build_runs composition the reference's jobs
perform (see skv.jobs for the job-level stream assembly). There is no CPU mode: if the
library or the GPU is missing this raises, it never falls back.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import List, Optional, Sequence, Tuple

from ._abi import (
    EXPORTED_SYMBOLS,
    LIB_PATH,
    PKG_DIR,
    SKV_OK,
    OutRun,
    RunError,
    SkvResult,
    SkvTimings,
    StreamArgs,
    result_to_runs,
)

MAX_RUN_SIZE = 4 * 1024 * 1024  # the jobs' build_runs limit (table_buffer_compaction.rs:103)

_lib = None


def build(force: bool = False) -> str:
    """Compile skv/libskv.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    src_dir = os.path.dirname(PKG_DIR)
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", src_dir] + (["-B"] if force else []))
    return LIB_PATH


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is not built (run skv.api.build() / __graft_entry__.build())")
    l = C.CDLL(LIB_PATH)
    l.skv_abi_version.restype = C.c_int
    l.skv_device_count.argtypes = [C.POINTER(C.c_int)]
    l.skv_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    l.skv_ctx_destroy.argtypes = [C.c_void_p]
    l.skv_ctx_destroy.restype = None
    l.skv_last_error.argtypes = [C.c_void_p]
    l.skv_last_error.restype = C.c_char_p
    l.skv_ctx_set_profiling.argtypes = [C.c_void_p, C.c_int]
    l.skv_ctx_get_timings.argtypes = [C.c_void_p, C.POINTER(SkvTimings)]
    l.skv_ctx_host_info.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    l.skv_ctx_host_info.restype = C.c_int
    l.skv_host_plan.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                C.POINTER(C.c_int), C.c_int]
    l.skv_host_plan.restype = C.c_int
    l.skv_split_deal.argtypes = [C.POINTER(C.c_int), C.c_uint32, C.c_uint64, C.POINTER(C.c_uint32),
                                 C.POINTER(C.c_int64)]
    l.skv_split_deal.restype = C.c_int
    l.skv_test_option.argtypes = [C.c_char_p, C.c_char_p]
    l.skv_test_option.restype = C.c_int
    for fn in (l.skv_compact, l.skv_compact_dev):
        fn.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32, C.POINTER(C.POINTER(SkvResult))]
        fn.restype = C.c_int
    l.skv_compact_split.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32,
                                    C.POINTER(C.POINTER(SkvResult))]
    l.skv_compact_split.restype = C.c_int
    l.skv_search_run.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32,
                                 C.c_void_p]
    l.skv_search_run.restype = C.c_int
    l.skv_run_index_create.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]
    l.skv_run_index_create.restype = C.c_int
    l.skv_run_index_search.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]
    l.skv_run_index_search.restype = C.c_int
    l.skv_run_index_free.argtypes = [C.c_void_p]
    l.skv_run_index_free.restype = None
    for fn in (l.skv_scan_runs, l.skv_scan_runs_dev):
        fn.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint64,
                       C.POINTER(C.POINTER(SkvResult))]
        fn.restype = C.c_int
    for fn in (l.skv_encode_batch, l.skv_encode_batch_dev):
        fn.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(C.POINTER(SkvResult))]
        fn.restype = C.c_int
    l.skv_result_free.argtypes = [C.POINTER(SkvResult)]
    l.skv_result_free.restype = None
    _lib = l
    return l


def exported_symbols_present() -> List[str]:
    l = load()
    return [s for s in EXPORTED_SYMBOLS if hasattr(l, s)]


class DeviceResult:
    """Output of compact_dev: run bytes stay in HBM (device pointer owned by the ctx)."""

    def __init__(self, lib, res_ptr, owner=None):
        self._lib = lib
        self._res = res_ptr
        # the bytes live in the ctx's "out" buffer: keep the Compactor (and so the ctx) alive
        # while this result is (skv.h: valid until the next call on the ctx or skv_result_free)
        self._owner = owner
        r = res_ptr.contents
        self.dev_ptr = int(r.bytes or 0)
        self.n_bytes = int(r.n_bytes)
        self.n_runs = int(r.n_runs)
        self.in_bytes = int(r.in_bytes)
        self.in_records = int(r.in_records)
        self.out_records = int(r.out_records)
        self._descs = None

    @property
    def descs(self):
        """Run descriptors as tuples (built on first use: a hot loop that only needs the byte
        counts does not pay for 1000+ ctypes reads)."""
        if self._descs is None:
            r = self._res.contents
            self._descs = [(d.off, d.len, d.put_count, d.delete_count, d.min_key_off, d.min_key_len, d.max_key_off,
                            d.max_key_len, d.table_id) for d in (r.runs[i] for i in range(r.n_runs))]
        return self._descs

    def free(self):
        if self._res:
            self._lib.skv_result_free(self._res)
            self._res = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class HostResult(DeviceResult):
    """Output of skv_compact (host inputs): the run bytes are in pinned host memory owned by the
    result (skv_result_free gives them back to the ctx's pool)."""

    def host_bytes(self, start: int = 0, length: Optional[int] = None):
        """A numpy view of output bytes [start, start + length) -- valid until free()."""
        import numpy as np

        n = self.n_bytes - start if length is None else length
        assert 0 <= start and start + n <= self.n_bytes
        if n == 0:
            return np.empty(0, dtype=np.uint8)
        return np.ctypeslib.as_array((C.c_uint8 * n).from_address(self.dev_ptr + start))


class Compactor:
    def __init__(self, device: int = 0, profiling: bool = False):
        self.lib = load()
        self.ctx = C.c_void_p()
        rc = self.lib.skv_ctx_create(device, C.byref(self.ctx))
        if rc != SKV_OK:
            raise RunError(rc, f"skv_ctx_create(device={device}) failed: no usable HIP device")
        if profiling:
            self.lib.skv_ctx_set_profiling(self.ctx, 1)

    def close(self):
        if self.ctx:
            self.lib.skv_ctx_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def host_info(self) -> dict:
        """skv_ctx_host_info: the NUMA node of this ctx's GPU (-1: unknown) and its host pool's threads."""
        node, threads = C.c_int(-1), C.c_int(0)
        rc = self.lib.skv_ctx_host_info(self.ctx, C.byref(node), C.byref(threads))
        if rc != SKV_OK:
            raise self._err(rc)
        return {"numa_node": node.value, "host_threads": threads.value}

    def _err(self, rc):
        return RunError(rc, self.lib.skv_last_error(self.ctx).decode("utf-8", "replace"))

    def compact(self, streams: Sequence[Tuple[int, Sequence[bytes]]], max_run_size: int = MAX_RUN_SIZE,
                flags: int = 0, with_info: bool = False):
        """streams: [(seq_no, [run_bytes, ...])] (host memory). Returns [OutRun]."""
        sa = StreamArgs(streams)
        res = C.POINTER(SkvResult)()
        rc = self.lib.skv_compact(self.ctx, sa.ptr, sa.n, max_run_size, flags, C.byref(res))
        if rc != SKV_OK:
            raise self._err(rc)
        try:
            runs = result_to_runs(res.contents)
            info = dict(in_bytes=res.contents.in_bytes, in_records=res.contents.in_records,
                        out_records=res.contents.out_records, dropped_tables=res.contents.dropped_tables,
                        n_bytes=res.contents.n_bytes)
        finally:
            self.lib.skv_result_free(res)
        return (runs, info) if with_info else runs

    def compact_dev(self, streams, max_run_size: int = MAX_RUN_SIZE, flags: int = 0) -> DeviceResult:
        """streams: [(seq_no, [(device_ptr, length), ...])] with inputs resident in HBM, or a
        StreamArgs(..., device=True) built once and reused (the caller's skv_stream[] table)."""
        sa = streams if isinstance(streams, StreamArgs) else StreamArgs(streams, device=True)
        res = C.POINTER(SkvResult)()
        rc = self.lib.skv_compact_dev(self.ctx, sa.ptr, sa.n, max_run_size, flags, C.byref(res))
        if rc != SKV_OK:
            raise self._err(rc)
        return DeviceResult(self.lib, res, self)

    def compact_host_ptrs(self, streams: Sequence[Tuple[int, Sequence[Tuple[int, int]]]],
                          max_run_size: int = MAX_RUN_SIZE, flags: int = 0, with_runs: bool = False):
        """skv_compact on raw host buffers (e.g. pinned tensors): [(seq_no, [(host_ptr, length)])].
        Returns (output bytes, output runs) -- or, with_runs, the [OutRun] -- and releases the pinned
        output. streams may also be a StreamArgs built with device=True (a table reused across calls)."""
        sa = streams if isinstance(streams, StreamArgs) else StreamArgs(streams, device=True)
        res = C.POINTER(SkvResult)()
        rc = self.lib.skv_compact(self.ctx, sa.ptr, sa.n, max_run_size, flags, C.byref(res))
        if rc != SKV_OK:
            raise self._err(rc)
        try:
            if with_runs:
                return result_to_runs(res.contents)
            return (int(res.contents.n_bytes), int(res.contents.n_runs))
        finally:
            self.lib.skv_result_free(res)

    def compact_host(self, streams, max_run_size: int = MAX_RUN_SIZE, flags: int = 0) -> HostResult:
        """skv_compact on raw host buffers ([(seq_no, [(host_ptr, length)])] or a StreamArgs built
        with device=True), keeping the result: bytes in pinned host memory plus the descriptors."""
        sa = streams if isinstance(streams, StreamArgs) else StreamArgs(streams, device=True)
        res = C.POINTER(SkvResult)()
        rc = self.lib.skv_compact(self.ctx, sa.ptr, sa.n, max_run_size, flags, C.byref(res))
        if rc != SKV_OK:
            raise self._err(rc)
        return HostResult(self.lib, res, self)

    def encode_batch(self, ops_run: bytes, max_run_size: int = MAX_RUN_SIZE, with_info: bool = False):
        """Writer batch encode (writer_service.rs:148-162): ops_run = the batch's ops in request
        order as one v1 run; returns build_runs over the ops sorted by key, last op per key kept."""
        buf = C.create_string_buffer(bytes(ops_run), max(1, len(ops_run)))
        res = C.POINTER(SkvResult)()
        rc = self.lib.skv_encode_batch(self.ctx, C.cast(buf, C.c_void_p), len(ops_run), max_run_size, C.byref(res))
        if rc != SKV_OK:
            raise self._err(rc)
        try:
            runs = result_to_runs(res.contents)
            info = dict(in_bytes=res.contents.in_bytes, in_records=res.contents.in_records,
                        out_records=res.contents.out_records)
        finally:
            self.lib.skv_result_free(res)
        return (runs, info) if with_info else runs

    def encode_batch_dev(self, ptr: int, length: int, max_run_size: int = MAX_RUN_SIZE) -> DeviceResult:
        """skv_encode_batch_dev: the ops run already in HBM."""
        res = C.POINTER(SkvResult)()
        rc = self.lib.skv_encode_batch_dev(self.ctx, C.c_void_p(ptr), length, max_run_size, C.byref(res))
        if rc != SKV_OK:
            raise self._err(rc)
        return DeviceResult(self.lib, res, self)

    def run_index(self, run: bytes) -> "RunIndex":
        """skv_run_index_create: the run staged and parsed once for many lookup batches."""
        run = bytes(run)
        buf = C.create_string_buffer(run, max(1, len(run)))
        h = C.c_void_p()
        rc = self.lib.skv_run_index_create(self.ctx, C.cast(buf, C.c_void_p), len(run), C.byref(h))
        if rc != SKV_OK:
            raise self._err(rc)
        return RunIndex(self, h, run)

    def _lookup(self, fn, run: bytes, keys: Sequence[bytes]):
        import numpy as np

        from ._abi import LOOKUP_FOUND, LOOKUP_NOT_FOUND, LOOKUP_TOMBSTONE, PANIC_TEXT, SkvLookup

        kb = b"".join(bytes(k) for k in keys)
        offs = np.zeros(len(keys) + 1, dtype=np.uint64)
        if keys:
            offs[1:] = np.cumsum([len(k) for k in keys])
        qbuf = C.create_string_buffer(kb, max(1, len(kb)))
        out = (SkvLookup * max(1, len(keys)))()
        rc = fn(C.cast(qbuf, C.c_void_p), C.c_void_p(offs.ctypes.data), len(keys), C.cast(out, C.c_void_p))
        if rc not in (SKV_OK, 4):  # 4 = SKV_E_FORMAT: some key panicked, outcomes filled in
            raise self._err(rc)
        res = []
        for i in range(len(keys)):
            o = out[i]
            if o.kind == LOOKUP_FOUND:
                res.append(("found", run[o.val_off:o.val_off + o.val_len]))
            elif o.kind == LOOKUP_TOMBSTONE:
                res.append(("tombstone", None))
            elif o.kind == LOOKUP_NOT_FOUND:
                res.append(("not_found", None))
            else:
                res.append(("panic", PANIC_TEXT[o.panic & 0xFF].format(o.panic >> 8)))
        return res

    def search_run(self, run: bytes, keys: Sequence[bytes]):
        """runs::search_run (runs.rs:285-398) for every key at once on the device. Returns one
        outcome per key: ("found", value) | ("tombstone", None) | ("not_found", None) |
        ("panic", reference panic text)."""
        import numpy as np

        from ._abi import (LOOKUP_FOUND, LOOKUP_NOT_FOUND, LOOKUP_PANIC, LOOKUP_TOMBSTONE, PANIC_TEXT,
                           SkvLookup)

        run = bytes(run)
        kb = b"".join(bytes(k) for k in keys)
        offs = np.zeros(len(keys) + 1, dtype=np.uint64)
        if keys:
            offs[1:] = np.cumsum([len(k) for k in keys])
        rbuf = C.create_string_buffer(run, max(1, len(run)))
        qbuf = C.create_string_buffer(kb, max(1, len(kb)))
        out = (SkvLookup * max(1, len(keys)))()
        rc = self.lib.skv_search_run(self.ctx, C.cast(rbuf, C.c_void_p), len(run), C.cast(qbuf, C.c_void_p),
                                     C.c_void_p(offs.ctypes.data), len(keys), C.cast(out, C.c_void_p))
        if rc not in (SKV_OK, 4):  # 4 = SKV_E_FORMAT: some key panicked, outcomes filled in
            raise self._err(rc)
        res = []
        for i in range(len(keys)):
            o = out[i]
            if o.kind == LOOKUP_FOUND:
                res.append(("found", run[o.val_off:o.val_off + o.val_len]))
            elif o.kind == LOOKUP_TOMBSTONE:
                res.append(("tombstone", None))
            elif o.kind == LOOKUP_NOT_FOUND:
                res.append(("not_found", None))
            else:
                assert o.kind == LOOKUP_PANIC
                res.append(("panic", PANIC_TEXT[o.panic & 0xFF].format(o.panic >> 8)))
        return res

    def scan_runs(self, runs: Sequence[bytes], exclusive_start_key: bytes, max_results: int):
        """ScanFromRun (cache_service.rs:97-151) over fetched runs on the device: the response items
        as one v1 run ([OutRun], [] when there is no item). Raises RunError: SKV_E_INVALID_ARG for
        max_results outside 1..=10000, or the merge error the reader reaches (read_run_iter text)."""
        bufs = [C.create_string_buffer(bytes(r), max(1, len(r))) for r in runs]
        ptrs = (C.c_void_p * max(1, len(runs)))(*[C.cast(b, C.c_void_p) for b in bufs])
        lens = (C.c_uint64 * max(1, len(runs)))(*[len(r) for r in runs])
        sk = C.create_string_buffer(bytes(exclusive_start_key), max(1, len(exclusive_start_key)))
        res = C.POINTER(SkvResult)()
        rc = self.lib.skv_scan_runs(self.ctx, C.cast(ptrs, C.c_void_p), C.cast(lens, C.c_void_p), len(runs),
                                    C.cast(sk, C.c_void_p), len(exclusive_start_key), max_results, C.byref(res))
        if rc != SKV_OK:
            raise self._err(rc)
        try:
            return result_to_runs(res.contents)
        finally:
            self.lib.skv_result_free(res)

    def timings(self) -> dict:
        t = SkvTimings()
        self.lib.skv_ctx_get_timings(self.ctx, C.byref(t))
        return {f: getattr(t, f) for f, _ in SkvTimings._fields_}


def compact_split(compactors: Sequence["Compactor"], streams, max_run_size: int = MAX_RUN_SIZE, flags: int = 0,
                  keep: bool = False, with_info: bool = False):
    """skv_compact_split: one compaction spread over the Compactors' GPUs by key range (the first
    one owns the result and reports errors). streams: [(seq_no, [run_bytes, ...])] (host memory),
    [(seq_no, [(host_ptr, length)])] or a StreamArgs built with device=True. Returns [OutRun] (with
    with_info, ([OutRun], info) as Compactor.compact), or, keep=True, the HostResult."""
    if not compactors:
        raise ValueError("compact_split needs at least one Compactor")
    home = compactors[0]
    if isinstance(streams, StreamArgs):
        sa = streams
    elif streams and streams[0][1] and isinstance(streams[0][1][0], tuple):
        sa = StreamArgs(streams, device=True)
    else:
        sa = StreamArgs(streams)
    ctxs = (C.c_void_p * len(compactors))(*[c.ctx.value for c in compactors])
    res = C.POINTER(SkvResult)()
    rc = home.lib.skv_compact_split(ctxs, len(compactors), sa.ptr, sa.n, max_run_size, flags, C.byref(res))
    if rc != SKV_OK:
        raise home._err(rc)
    if keep:
        return HostResult(home.lib, res, home)
    try:
        runs = result_to_runs(res.contents)
        info = dict(in_bytes=res.contents.in_bytes, in_records=res.contents.in_records,
                    out_records=res.contents.out_records, dropped_tables=res.contents.dropped_tables,
                    n_bytes=res.contents.n_bytes)
    finally:
        home.lib.skv_result_free(res)
    return (runs, info) if with_info else runs


class RunIndex:
    """A run parsed once (skv_run_index_create); search() takes any number of lookup batches."""

    def __init__(self, owner: Compactor, handle, run: bytes):
        self._owner = owner  # the ctx the index was built with (same device) stays alive
        self._h = handle
        self._run = run

    def search(self, keys: Sequence[bytes]):
        lib, ctx, h = self._owner.lib, self._owner.ctx, self._h
        return self._owner._lookup(lambda q, o, n, out: lib.skv_run_index_search(ctx, h, q, o, n, out), self._run,
                                   keys)

    def close(self):
        if self._h:
            self._owner.lib.skv_run_index_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def device_count() -> int:
    n = C.c_int(0)
    load().skv_device_count(C.byref(n))
    return n.value


def host_plan(pci_bus_id: str, n_devices: int, hw_threads: int, sysfs_root: str = "/sys") -> dict:
    """skv_host_plan: the NUMA node, host-pool size and CPUs the library gives the GPU at `pci_bus_id`
    (no device needed; a stub sysfs tree may stand in for /sys)."""
    l = load()
    node, threads = C.c_int(-1), C.c_int(0)
    cpus = (C.c_int * 4096)()
    n = l.skv_host_plan(sysfs_root.encode(), pci_bus_id.encode(), n_devices, hw_threads, C.byref(node),
                        C.byref(threads), cpus, 4096)
    return {"numa_node": node.value, "pool_threads": threads.value, "cpus": sorted(cpus[:max(n, 0)])}


def split_deal(ctx_devices: Sequence[int], n_parts: int) -> tuple:
    """skv_split_deal: (ctx of each part, the part whose H2D each part waits for or -1) for
    skv_compact_split over ctxs on the devices `ctx_devices` (no device needed)."""
    l = load()
    g = len(ctx_devices)
    dev = (C.c_int * g)(*ctx_devices)
    ctx_of = (C.c_uint32 * max(n_parts, 1))()
    after = (C.c_int64 * max(n_parts, 1))()
    rc = l.skv_split_deal(dev, g, n_parts, ctx_of, after)
    if rc != SKV_OK:
        raise RunError(rc, "skv_split_deal: invalid arguments")
    return list(ctx_of[:n_parts]), list(after[:n_parts])


_test_opts: dict = {}


def test_option(name: Optional[str], value=None) -> None:
    """skv_test_option: set (value: str / int) or clear (None) one of the library's test hooks (tests
    only, include/skv.h); name None clears every hook."""
    l = load()
    rc = l.skv_test_option(name.encode() if name is not None else None,
                           str(value).encode() if value is not None else None)
    if rc != SKV_OK:
        raise RunError(rc, f"skv_test_option: unknown hook {name!r}")
    if name is None:
        _test_opts.clear()
    elif value is None:
        _test_opts.pop(name, None)
    else:
        _test_opts[name] = str(value)


def test_option_get(name: str) -> Optional[str]:
    """the value this process set for a test hook through test_option (None: unset)"""
    return _test_opts.get(name)
