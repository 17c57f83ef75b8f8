"""ctypes wrapper of oracle/libskv_oracle.so — the CPU restatement of skyvault's compaction
path. TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package (skyvault-rs_amd/skv).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
from typing import List, Sequence, Tuple

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "skyvault-rs_amd"))

from skv._abi import (  # noqa: E402
    SKV_OK,
    RunError,
    SkvResult,
    StreamArgs,
    result_to_runs,
)

LIB = os.path.join(HERE, "libskv_oracle.so")


class SkvoOp(C.Structure):
    _fields_ = [
        ("is_put", C.c_uint32),
        ("key_len", C.c_uint32),
        ("key", C.c_void_p),
        ("val_len", C.c_uint64),
        ("val", C.c_void_p),
    ]


class SkvoOpList(C.Structure):
    _fields_ = [("ops", C.POINTER(SkvoOp)), ("n_ops", C.c_uint64), ("arena", C.c_void_p)]


_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", HERE, "libskv_oracle.so"])
    return LIB


def lib():
    global _lib
    if _lib is None:
        build()
        l = C.CDLL(LIB)
        l.skvo_compact.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32,
                                   C.POINTER(C.POINTER(SkvResult)), C.c_char_p, C.c_size_t]
        l.skvo_compact.restype = C.c_int
        l.skvo_build_runs.argtypes = [C.POINTER(SkvoOp), C.c_uint64, C.c_uint64,
                                      C.POINTER(C.POINTER(SkvResult)), C.c_char_p, C.c_size_t]
        l.skvo_build_runs.restype = C.c_int
        l.skvo_decode_run.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.POINTER(SkvoOpList)),
                                      C.c_char_p, C.c_size_t]
        l.skvo_decode_run.restype = C.c_int
        l.skvo_merge_ops.argtypes = [C.POINTER(C.POINTER(SkvoOp)), C.POINTER(C.c_uint64),
                                     C.POINTER(C.c_int64), C.c_uint32,
                                     C.POINTER(C.POINTER(SkvoOpList)), C.c_char_p, C.c_size_t]
        l.skvo_merge_ops.restype = C.c_int
        l.skvo_scan_runs.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_uint64,
                                     C.POINTER(C.POINTER(SkvResult)), C.c_char_p, C.c_size_t]
        l.skvo_scan_runs.restype = C.c_int
        l.skvo_result_free.argtypes = [C.POINTER(SkvResult)]
        l.skvo_op_list_free.argtypes = [C.POINTER(SkvoOpList)]
        l.skvo_sb_new.argtypes = [C.c_uint64]
        l.skvo_sb_new.restype = C.c_void_p
        l.skvo_sb_feed_run.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_char_p, C.c_size_t]
        l.skvo_sb_feed_run.restype = C.c_int
        l.skvo_sb_pending.argtypes = [C.c_void_p]
        l.skvo_sb_pending.restype = C.c_uint64
        l.skvo_sb_drain.argtypes = [C.c_void_p, C.c_void_p]
        l.skvo_sb_drain.restype = None
        l.skvo_sb_finish.argtypes = [C.c_void_p, C.POINTER(C.POINTER(SkvResult))]
        l.skvo_sb_finish.restype = C.c_int
        l.skvo_sb_free.argtypes = [C.c_void_p]
        l.skvo_sb_free.restype = None
        _lib = l
    return _lib


# ops are tuples: (True, key_bytes, value_bytes) for Put, (False, key_bytes, None) for Delete
Op = Tuple[bool, bytes, object]


def _ops_array(ops: Sequence[Op]):
    keep = []
    arr = (SkvoOp * max(1, len(ops)))()
    for i, (is_put, k, v) in enumerate(ops):
        kb = C.create_string_buffer(bytes(k), max(1, len(k)))
        keep.append(kb)
        arr[i].is_put = 1 if is_put else 0
        arr[i].key_len = len(k)
        arr[i].key = C.cast(kb, C.c_void_p)
        if is_put:
            vb = C.create_string_buffer(bytes(v), max(1, len(v)))
            keep.append(vb)
            arr[i].val_len = len(v)
            arr[i].val = C.cast(vb, C.c_void_p)
    return arr, keep


def _op_list(ptr) -> List[Op]:
    l = ptr.contents
    out = []
    for i in range(l.n_ops):
        o = l.ops[i]
        k = C.string_at(o.key, o.key_len) if o.key_len else b""
        if o.is_put:
            v = C.string_at(o.val, o.val_len) if o.val_len else b""
            out.append((True, k, v))
        else:
            out.append((False, k, None))
    return out


def scan_runs(runs: Sequence[bytes], start_key: bytes, max_results: int):
    """ScanFromRun (cache_service.rs:97-151) over fetched runs: the response items as one v1 run
    ([OutRun], empty when there is no item), or RunError (the reference wraps it as
    Status::internal("Merge stream error: {e}")) / SKV_E_INVALID_ARG for max_results."""
    bufs = [C.create_string_buffer(bytes(r), max(1, len(r))) for r in runs]
    ptrs = (C.c_void_p * max(1, len(runs)))(*[C.cast(b, C.c_void_p) for b in bufs])
    lens = (C.c_uint64 * max(1, len(runs)))(*[len(r) for r in runs])
    sk = C.create_string_buffer(bytes(start_key), max(1, len(start_key)))
    res = C.POINTER(SkvResult)()
    eb = C.create_string_buffer(512)
    rc = lib().skvo_scan_runs(C.cast(ptrs, C.c_void_p), C.cast(lens, C.c_void_p), len(runs), C.cast(sk, C.c_void_p),
                              len(start_key), max_results, C.byref(res), eb, 512)
    if rc != SKV_OK:
        raise RunError(rc, eb.value.decode("utf-8", "replace"))
    try:
        return result_to_runs(res.contents)
    finally:
        lib().skvo_result_free(res)


def compact(streams: Sequence[tuple], max_run_size: int, flags: int = 0, with_result: bool = False):
    """streams: [(seq_no, [run_bytes, ...])]. Returns [OutRun] or raises RunError."""
    sa = StreamArgs(streams)
    res = C.POINTER(SkvResult)()
    eb = C.create_string_buffer(512)
    rc = lib().skvo_compact(sa.ptr, sa.n, max_run_size, flags, C.byref(res), eb, 512)
    if rc != SKV_OK:
        raise RunError(rc, eb.value.decode("utf-8", "replace"))
    try:
        runs = result_to_runs(res.contents)
        info = dict(in_bytes=res.contents.in_bytes, out_records=res.contents.out_records,
                    dropped_tables=res.contents.dropped_tables, n_bytes=res.contents.n_bytes)
    finally:
        lib().skvo_result_free(res)
    return (runs, info) if with_result else runs


def compact_bytes(streams: Sequence[tuple], max_run_size: int, flags: int = 0):
    """Like compact() but returns (concatenated output bytes, [descriptor tuples])."""
    sa = StreamArgs(streams)
    res = C.POINTER(SkvResult)()
    eb = C.create_string_buffer(512)
    rc = lib().skvo_compact(sa.ptr, sa.n, max_run_size, flags, C.byref(res), eb, 512)
    if rc != SKV_OK:
        raise RunError(rc, eb.value.decode("utf-8", "replace"))
    try:
        r = res.contents
        data = C.string_at(r.bytes, r.n_bytes) if r.n_bytes else b""
        descs = [(d.off, d.len, d.put_count, d.delete_count, d.min_key_off, d.min_key_len,
                  d.max_key_off, d.max_key_len, d.table_id) for d in (r.runs[i] for i in range(r.n_runs))]
    finally:
        lib().skvo_result_free(res)
    return data, descs


def build_runs(ops: Sequence[Op], max_run_size: int):
    arr, keep = _ops_array(ops)
    res = C.POINTER(SkvResult)()
    eb = C.create_string_buffer(512)
    rc = lib().skvo_build_runs(arr, len(ops), max_run_size, C.byref(res), eb, 512)
    if rc != SKV_OK:
        raise RunError(rc, eb.value.decode("utf-8", "replace"))
    try:
        return result_to_runs(res.contents)
    finally:
        lib().skvo_result_free(res)


def decode_run(data: bytes):
    """read_run_stream: returns (ops, error_or_None)."""
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    out = C.POINTER(SkvoOpList)()
    eb = C.create_string_buffer(512)
    rc = lib().skvo_decode_run(C.cast(buf, C.c_void_p), len(data), C.byref(out), eb, 512)
    try:
        ops = _op_list(out)
    finally:
        lib().skvo_op_list_free(out)
    err = None if rc == SKV_OK else RunError(rc, eb.value.decode("utf-8", "replace"))
    return ops, err


def merge_ops(streams: Sequence[Tuple[int, Sequence[Op]]]):
    """k_way::merge over decoded op lists: returns (emitted ops, error_or_None)."""
    n = len(streams)
    keep = []
    ptrs = (C.POINTER(SkvoOp) * max(1, n))()
    lens = (C.c_uint64 * max(1, n))()
    seqs = (C.c_int64 * max(1, n))()
    for i, (seq, ops) in enumerate(streams):
        arr, k = _ops_array(ops)
        keep += [arr, k]
        ptrs[i] = C.cast(arr, C.POINTER(SkvoOp))
        lens[i] = len(ops)
        seqs[i] = seq
    out = C.POINTER(SkvoOpList)()
    eb = C.create_string_buffer(512)
    rc = lib().skvo_merge_ops(ptrs, lens, seqs, n, C.byref(out), eb, 512)
    ops = []
    if out:
        try:
            ops = _op_list(out)
        finally:
            lib().skvo_op_list_free(out)
    err = None if rc == SKV_OK else RunError(rc, eb.value.decode("utf-8", "replace"))
    return ops, err


def encode_batch(ops_run: bytes, max_run_size: int):
    """writer_service.rs:148-162 (process_batch), restated: the batch's ops (decoded with the
    oracle's read_run_stream, oracle/skv_oracle.c) collected into a BTreeMap keyed by key — a
    later op replaces an earlier one of the same key — then build_runs over the map's values in
    key order. Returns (runs) or raises like compact()."""
    ops, err = decode_run(ops_run)
    if err is not None:  # one stream: its decode error always surfaces (k_way.rs:134-137, :154-171)
        raise err
    latest = {}
    for op in ops:
        latest[op[1]] = op
    return build_runs([latest[k] for k in sorted(latest)], max_run_size)


def search_run(run: bytes, key: bytes):
    """runs::search_run (runs.rs:285-398), restated literally (test infrastructure): scan from the
    first record; stop at the first key not below `key`. Returns ("found", value) |
    ("tombstone", None) | ("not_found", None) | ("panic", the reference's panic text)."""
    n = len(run)
    if n == 0:
        return ("panic", "Empty run data")  # :289-291
    if run[0] != 1:
        return ("panic", f"Unsupported version: {run[0]}")  # :294-297
    p = 1
    while p < n:  # :300
        m = run[p]
        p += 1
        if m not in (1, 2):
            return ("panic", f"Invalid marker byte: {m}")  # :307-310
        if p + 4 > n:
            return ("panic", "Incomplete key length data")  # :313-315
        klen = int.from_bytes(run[p:p + 4], "big")
        p += 4
        if p + klen > n:
            return ("panic", "Incomplete key data")  # :324-326
        k = run[p:p + klen]
        p += klen
        if k < key:  # :331-356
            if m == 1:
                if p + 4 > n:
                    return ("panic", "Incomplete value length data")
                vlen = int.from_bytes(run[p:p + 4], "big")
                p += 4
                if p + vlen > n:
                    return ("panic", "Incomplete value data")
                p += vlen
            continue
        if k == key:  # :357-386
            if m == 2:
                return ("tombstone", None)
            if p + 4 > n:
                return ("panic", "Incomplete value length data for found key")
            vlen = int.from_bytes(run[p:p + 4], "big")
            p += 4
            if p + vlen > n:
                return ("panic", "Incomplete value data for found key")
            return ("found", run[p:p + vlen])
        return ("not_found", None)  # :387-391
    return ("not_found", None)  # :395-396


class StreamBuilder:
    """Streaming runs::build_runs (runs.rs:166-282) over a merged op sequence that arrives as
    consecutive v1 runs (skvo_sb_* in skv_oracle.c): feed(run) -> the output bytes it
    completed; finish() -> (tail bytes, [descriptor tuples]) with absolute offsets. Used by the
    full-size tests, which merge key ranges separately with an unbounded max and split here."""

    def __init__(self, max_run_size: int):
        self._l = lib()
        self._s = self._l.skvo_sb_new(max_run_size)

    def feed(self, run, length: int = None) -> "np.ndarray":
        import numpy as np

        if isinstance(run, int):
            ptr, n = run, length
        else:
            a = np.frombuffer(run, dtype=np.uint8) if not isinstance(run, np.ndarray) else run
            ptr, n = a.ctypes.data, a.size
        eb = C.create_string_buffer(512)
        rc = self._l.skvo_sb_feed_run(self._s, C.c_void_p(ptr), n, eb, 512)
        if rc != SKV_OK:
            raise RunError(rc, eb.value.decode("utf-8", "replace"))
        out = np.empty(self._l.skvo_sb_pending(self._s), dtype=np.uint8)
        self._l.skvo_sb_drain(self._s, C.c_void_p(out.ctypes.data))
        return out

    def finish(self):
        res = C.POINTER(SkvResult)()
        rc = self._l.skvo_sb_finish(self._s, C.byref(res))
        if rc != SKV_OK:
            raise RunError(rc, "stream builder failed earlier")
        try:
            r = res.contents
            tail = C.string_at(r.bytes, r.n_bytes) if r.n_bytes else b""
            descs = [(d.off, d.len, d.put_count, d.delete_count, d.min_key_off, d.min_key_len,
                      d.max_key_off, d.max_key_len, d.table_id) for d in (r.runs[i] for i in range(r.n_runs))]
        finally:
            self._l.skvo_result_free(res)
        return tail, descs

    def __del__(self):
        try:
            if self._s:
                self._l.skvo_sb_free(self._s)
                self._s = None
        except Exception:
            pass


def compact_np(sa, max_run_size: int, flags: int = 0):
    """skvo_compact over a prebuilt skv_stream[] (skv._abi.StreamArgs / stream_table, host
    pointers). Returns (output bytes as a numpy array, [descriptor tuples], info dict) or
    raises RunError. For GiB-scale checks: no Python object per record or per stream."""
    import numpy as np

    res = C.POINTER(SkvResult)()
    eb = C.create_string_buffer(512)
    rc = lib().skvo_compact(sa.ptr, sa.n, max_run_size, flags, C.byref(res), eb, 512)
    if rc != SKV_OK:
        raise RunError(rc, eb.value.decode("utf-8", "replace"))
    try:
        r = res.contents
        data = np.empty(r.n_bytes, dtype=np.uint8)
        if r.n_bytes:
            C.memmove(data.ctypes.data, r.bytes, r.n_bytes)
        descs = [(d.off, d.len, d.put_count, d.delete_count, d.min_key_off, d.min_key_len,
                  d.max_key_off, d.max_key_len, d.table_id) for d in (r.runs[i] for i in range(r.n_runs))]
        info = dict(in_bytes=r.in_bytes, out_records=r.out_records, dropped_tables=r.dropped_tables)
    finally:
        lib().skvo_result_free(res)
    return data, descs, info
