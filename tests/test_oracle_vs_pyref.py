"""The C restatement (oracle/) and the independent Python restatement (tests/pyref.py) must
agree on every generated input: outputs byte-for-byte, stats, and the first error (kind and
message) — including corrupted runs, unsorted streams, tombstone dropping and WAL splitting.
This mirrors the reference's proptest round-trip (runs.rs:643-772) with a wider domain."""
import random

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import pyref
from skv import format as fmt

ALPH = ["a", "b", "c", "ab", "abc", "b0", "zz", "é", "p" * 20, "p" * 20 + "x", "p" * 17, ""]


def _key(r: random.Random, wal: bool) -> str:
    k = "".join(r.choice(ALPH) for _ in range(r.randint(0, 3)))
    if wal:
        t = r.choice(["1", "2", "10", "-3", "7", "+7", "07"]) if r.random() < 0.97 else r.choice(["x", "", "9" * 20])
        return f"{t}.{k}" if r.random() < 0.98 else k
    return k


def _run(r: random.Random, wal: bool, sorted_ok: bool) -> bytes:
    keys = sorted({_key(r, wal).encode() for _ in range(r.randint(0, 12))})
    if not sorted_ok and len(keys) > 1:
        i = r.randrange(len(keys) - 1)
        keys[i], keys[i + 1] = keys[i + 1], keys[i]
    if r.random() < 0.1 and keys:
        keys.insert(r.randrange(len(keys)), r.choice(keys))  # in-stream duplicate
    ops = []
    for k in keys:
        if r.random() < 0.25:
            ops.append(fmt.delete(k))
        else:
            ops.append(fmt.put(k, bytes(r.getrandbits(8) for _ in range(r.randint(0, 9)))))
    data = bytearray(fmt.encode_run(ops))
    c = r.random()
    if c < 0.04:
        data = data[: r.randint(0, len(data))]
    elif c < 0.06 and len(data) > 1:
        data[r.randrange(1, len(data))] = r.getrandbits(8)
    elif c < 0.07:
        data[0:1] = bytes([r.choice([0, 2, 255])])
    elif c < 0.08:
        data += b"\x02\x00\x00\x00\x01\xff"
    return bytes(data)


def _case(seed: int):
    r = random.Random(seed)
    flags = r.choice([0, 0, 1, 2])
    wal = flags == 2
    sorted_ok = r.random() < 0.9
    n = r.randint(0, 6)
    seqs = r.sample(range(-5, 50), n)
    streams = []
    for s in seqs:
        members = [_run(r, wal, sorted_ok) for _ in range(r.choice([0, 1, 1, 1, 2, 3]))]
        streams.append((s, members))
    max_size = r.choice([0, 16, 40, 100, 1 << 22])
    return streams, max_size, flags


def _norm_oracle(oracle, streams, max_size, flags):
    try:
        runs, info = oracle.compact(streams, max_size, flags, with_result=True)
        return ("ok", [(r.data, r.stats.min_key.encode(), r.stats.max_key.encode(), r.stats.size_bytes,
                        r.stats.put_count, r.stats.delete_count, r.table_id) for r in runs], info["dropped_tables"])
    except Exception as e:
        return ("err", e.code, e.message)


def _norm_pyref(streams, max_size, flags):
    try:
        runs, dropped = pyref.compact(streams, max_size, flags)
        return ("ok", [(b, s[0], s[1], s[2], s[3], s[4], t) for b, s, t in runs], dropped)
    except pyref.Err as e:
        return ("err", e.code, e.msg)


@settings(max_examples=400, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.integers(min_value=0, max_value=2**32))
def test_oracle_matches_pyref(oracle, seed):
    streams, max_size, flags = _case(seed)
    assert _norm_oracle(oracle, streams, max_size, flags) == _norm_pyref(streams, max_size, flags)


def test_duplicate_seq_rejected(oracle):
    with pytest.raises(Exception) as ei:
        oracle.compact([(1, [b"\x01"]), (1, [b"\x01"])], 1 << 22)
    assert ei.value.code == 6
