"""ctypes mirror of include/skv.h (the C ABI of the compaction path).

Shared by the product wrapper (skv.runs / skv.jobs, which load libskv.so) and by the test
tooling that loads the CPU restatement under oracle/. Only plain pointers and sizes cross
the boundary — no torch types.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT_DIR = os.path.dirname(os.path.dirname(PKG_DIR))
# SKV_LIB selects an alternative build of the same library (tuning variants, tools/variants.sh)
LIB_PATH = os.environ.get("SKV_LIB") or os.path.join(PKG_DIR, "libskv.so")

SKV_OK = 0
SKV_E_EMPTY_INPUT = 1
SKV_E_UNSUPPORTED_VERSION = 2
SKV_E_IO = 3
SKV_E_FORMAT = 4
SKV_E_INVALID_INPUT = 5
SKV_E_INVALID_ARG = 6
SKV_E_DEVICE = 7
SKV_E_UNSUPPORTED = 8
SKV_E_INTERNAL = 9

SKV_DROP_TOMBSTONES = 1
SKV_SPLIT_BY_TABLE = 2

ERROR_NAMES = {
    SKV_E_EMPTY_INPUT: "EmptyInput",
    SKV_E_UNSUPPORTED_VERSION: "UnsupportedVersion",
    SKV_E_IO: "Io",
    SKV_E_FORMAT: "Format",
    SKV_E_INVALID_INPUT: "InvalidInput",
    SKV_E_INVALID_ARG: "InvalidArgument",
    SKV_E_DEVICE: "Device",
    SKV_E_UNSUPPORTED: "Unsupported",
    SKV_E_INTERNAL: "Internal",
}


class SkvStream(C.Structure):
    _fields_ = [
        ("runs", C.POINTER(C.c_void_p)),
        ("run_lens", C.POINTER(C.c_uint64)),
        ("n_runs", C.c_uint32),
        ("seq_no", C.c_int64),
    ]


class SkvRunDesc(C.Structure):
    _fields_ = [
        ("off", C.c_uint64),
        ("len", C.c_uint64),
        ("put_count", C.c_uint64),
        ("delete_count", C.c_uint64),
        ("min_key_off", C.c_uint64),
        ("min_key_len", C.c_uint64),
        ("max_key_off", C.c_uint64),
        ("max_key_len", C.c_uint64),
        ("table_id", C.c_int64),
        ("reserved", C.c_uint64),
    ]


class SkvResult(C.Structure):
    _fields_ = [
        ("bytes", C.c_void_p),
        ("n_bytes", C.c_uint64),
        ("runs", C.POINTER(SkvRunDesc)),
        ("n_runs", C.c_uint64),
        ("in_bytes", C.c_uint64),
        ("in_records", C.c_uint64),
        ("out_records", C.c_uint64),
        ("dropped_tables", C.c_uint64),
    ]


class SkvLookup(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("panic", C.c_uint32), ("val_off", C.c_uint64), ("val_len", C.c_uint64)]


LOOKUP_NOT_FOUND, LOOKUP_FOUND, LOOKUP_TOMBSTONE, LOOKUP_PANIC = 0, 1, 2, 3
PANIC_TEXT = {1: "Empty run data", 2: "Unsupported version: {}", 3: "Invalid marker byte: {}",
              4: "Incomplete key length data", 5: "Incomplete key data", 6: "Incomplete value length data",
              7: "Incomplete value data", 8: "Incomplete value length data for found key",
              9: "Incomplete value data for found key"}


class SkvTimings(C.Structure):
    _fields_ = [
        ("total_ms", C.c_double),
        ("parse_ms", C.c_double),
        ("check_ms", C.c_double),
        ("merge_ms", C.c_double),
        ("chain_ms", C.c_double),
        ("gather_ms", C.c_double),
        ("gather_read_bytes", C.c_uint64),
        ("gather_write_bytes", C.c_uint64),
        ("host_syncs", C.c_uint64),
        ("host_total_ms", C.c_double),
        ("host_sync_ms", C.c_double),
        ("path", C.c_uint32),
        ("fused_reject", C.c_uint32),
        ("hot_ms", C.c_double),
        ("hot_read_bytes", C.c_uint64),
        ("hot_write_bytes", C.c_uint64),
        ("sorted", C.c_uint32),
        ("fp_rerun", C.c_uint32),
        ("host_parts", C.c_uint32),
        ("span_parse", C.c_uint32),
        ("wal_stage", C.c_uint32),
        ("reserved2", C.c_uint32),
    ]


# skv_timings.path (include/skv.h)
PATH_GENERAL, PATH_FIXED, PATH_FUSED = 1, 2, 3
PATH_NAMES = {PATH_GENERAL: "general", PATH_FIXED: "fixed", PATH_FUSED: "fused"}


# Every symbol include/skv.h declares (tests/test_abi.py checks the built library exports them).
EXPORTED_SYMBOLS = [
    "skv_abi_version",
    "skv_device_count",
    "skv_ctx_create",
    "skv_ctx_destroy",
    "skv_last_error",
    "skv_ctx_set_profiling",
    "skv_ctx_get_timings",
    "skv_ctx_host_info",
    "skv_host_plan",
    "skv_split_deal",
    "skv_test_option",
    "skv_compact",
    "skv_compact_dev",
    "skv_compact_split",
    "skv_encode_batch",
    "skv_encode_batch_dev",
    "skv_search_run",
    "skv_run_index_create",
    "skv_run_index_search",
    "skv_run_index_free",
    "skv_scan_runs",
    "skv_scan_runs_dev",
    "skv_result_free",
]


@dataclass
class Stats:
    """Stats::StatsV1 (runs.rs:102-109)."""

    min_key: str
    max_key: str
    size_bytes: int
    put_count: int
    delete_count: int


@dataclass
class OutRun:
    data: bytes
    stats: Stats
    table_id: int = 0


class RunError(Exception):
    """RunError / JobError surfaced through the ABI. `kind` names the reference variant,
    `message` is the reference's Display text."""

    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code
        self.kind = ERROR_NAMES.get(code, str(code))
        self.message = message


def _stream_dtype():
    import numpy as np

    return np.dtype({"names": ["runs", "run_lens", "n_runs", "seq_no"],
                     "formats": [np.uint64, np.uint64, np.uint32, np.int64],
                     "offsets": [SkvStream.runs.offset, SkvStream.run_lens.offset, SkvStream.n_runs.offset,
                                 SkvStream.seq_no.offset],
                     "itemsize": C.sizeof(SkvStream)})


class StreamArgs:
    """Keeps the ctypes arrays of one skv_stream[] alive for a call."""

    def __init__(self, streams: Sequence[tuple], device: bool = False):
        # streams: [(seq_no, [run_ptr_or_bytes, ...], [len, ...]?)]
        self._keep: List[object] = []
        self.n = len(streams)
        if device:  # numpy-built tables: one flat pointer / length array + the stream structs
            import numpy as np

            counts = np.fromiter((len(st[1]) for st in streams), dtype=np.int64, count=len(streams))
            flat = [r for st in streams for r in st[1]]
            ptrs = np.array([int(p) for p, _ in flat] or [0], dtype=np.uint64)
            lens = np.array([int(l) for _, l in flat] or [0], dtype=np.uint64)
            offs = np.zeros(len(streams), dtype=np.uint64)
            if len(streams) > 1:
                offs[1:] = np.cumsum(counts[:-1]) * 8
            tbl = np.zeros(max(1, len(streams)), dtype=_STREAM_DT)
            tbl["runs"][: len(streams)] = ptrs.ctypes.data + offs
            tbl["run_lens"][: len(streams)] = lens.ctypes.data + offs
            tbl["n_runs"][: len(streams)] = counts
            tbl["seq_no"][: len(streams)] = [int(st[0]) for st in streams]
            self._keep += [ptrs, lens, tbl]
            self.ptr = C.c_void_p(tbl.ctypes.data)
            return
        self.arr = (SkvStream * max(1, len(streams)))()
        self.ptr = C.cast(self.arr, C.c_void_p)
        for i, st in enumerate(streams):
            seq, runs = st[0], st[1]
            n = len(runs)
            ptrs = (C.c_void_p * max(1, n))()
            lens = (C.c_uint64 * max(1, n))()
            for j, r in enumerate(runs):
                if device:
                    ptr, ln = r
                    ptrs[j] = C.c_void_p(int(ptr))
                    lens[j] = int(ln)
                else:
                    b = bytes(r)
                    buf = C.create_string_buffer(b, max(1, len(b)))
                    self._keep.append(buf)
                    ptrs[j] = C.cast(buf, C.c_void_p)
                    lens[j] = len(b)
            self._keep += [ptrs, lens]
            self.arr[i].runs = C.cast(ptrs, C.POINTER(C.c_void_p))
            self.arr[i].run_lens = C.cast(lens, C.POINTER(C.c_uint64))
            self.arr[i].n_runs = n
            self.arr[i].seq_no = int(seq)


_STREAM_DT = _stream_dtype()


def stream_table(seq_nos, run_ptrs, run_lens) -> StreamArgs:
    """skv_stream[] of one member run per stream straight from numpy arrays (no Python loop per
    stream): seq_nos int64, run_ptrs / run_lens uint64 (host or device addresses)."""
    import numpy as np

    seq = np.ascontiguousarray(seq_nos, dtype=np.int64)
    ptrs = np.ascontiguousarray(run_ptrs, dtype=np.uint64)
    lens = np.ascontiguousarray(run_lens, dtype=np.uint64)
    n = seq.size
    sa = StreamArgs.__new__(StreamArgs)
    tbl = np.zeros(max(1, n), dtype=_STREAM_DT)
    idx = np.arange(n, dtype=np.uint64) * np.uint64(8)
    tbl["runs"][:n] = np.uint64(ptrs.ctypes.data) + idx
    tbl["run_lens"][:n] = np.uint64(lens.ctypes.data) + idx
    tbl["n_runs"][:n] = 1
    tbl["seq_no"][:n] = seq
    sa._keep = [ptrs, lens, tbl]
    sa.n = n
    sa.ptr = C.c_void_p(tbl.ctypes.data)
    return sa


def result_to_runs(res: SkvResult, host_bytes: Optional[bytes] = None) -> List[OutRun]:
    """Turn an skv_result (host bytes) into [(run bytes, StatsV1)]."""
    if host_bytes is None:
        host_bytes = C.string_at(res.bytes, res.n_bytes) if res.n_bytes else b""
    out = []
    for i in range(res.n_runs):
        d = res.runs[i]
        data = host_bytes[d.off : d.off + d.len]
        mn = host_bytes[d.min_key_off : d.min_key_off + d.min_key_len].decode("utf-8")
        mx = host_bytes[d.max_key_off : d.max_key_off + d.max_key_len].decode("utf-8")
        out.append(OutRun(data, Stats(mn, mx, d.len, d.put_count, d.delete_count), d.table_id))
    return out
