"""Skyvault run format v1 (runs.rs:97-100, :240-267) — host-side writer and constants.

    run    := version:u8(=1) record*
    record := 0x01 key_len:u32be key val_len:u32be val      (Put,    runs.rs:253-259)
            | 0x02 key_len:u32be key                        (Delete, runs.rs:261-266)

The writer here only serialises an already-sorted op list into ONE run without size
splitting; it is what the synthetic workload generators and tests use to produce input
runs (the reference produces them with build_runs in the writer service,
writer_service.rs:148-171). Compaction itself happens on the GPU through the C ABI.
"""
from __future__ import annotations

import struct
from typing import Iterable, Tuple, Union

CURRENT_VERSION = 1
MARKER_PUT = 1
MARKER_DELETE = 2

KeyT = Union[str, bytes]


def _kb(k: KeyT) -> bytes:
    return k.encode("utf-8") if isinstance(k, str) else bytes(k)


def put(key: KeyT, value: bytes) -> Tuple[bool, bytes, bytes]:
    """WriteOperation::Put (runs.rs:41) as (is_put, key_bytes, value_bytes)."""
    return (True, _kb(key), bytes(value))


def delete(key: KeyT) -> Tuple[bool, bytes, None]:
    """WriteOperation::Delete (runs.rs:42)."""
    return (False, _kb(key), None)


def encode_record(op) -> bytes:
    is_put, k, v = op
    if is_put:
        return struct.pack(">BI", MARKER_PUT, len(k)) + k + struct.pack(">I", len(v)) + v
    return struct.pack(">BI", MARKER_DELETE, len(k)) + k


def encode_run(ops: Iterable) -> bytes:
    """version byte + records, no splitting, no order check (input generation only)."""
    return bytes([CURRENT_VERSION]) + b"".join(encode_record(o) for o in ops)


def op_size(op) -> int:
    """runs.rs:202-209"""
    is_put, k, v = op
    return 1 + 4 + len(k) + 4 + len(v) if is_put else 1 + 4 + len(k)
