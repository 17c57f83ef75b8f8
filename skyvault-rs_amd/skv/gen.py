"""Deterministic synthetic workloads for the BASELINE.json configs.

Every generator is a pure function of its seed (splitmix64, base seed 0x5EEDC0DE; stream s
uses base + s). Runs are produced in the v1 format with keys sorted and unique inside each
run, the shape build_runs emits (runs.rs:190-198). Vectorised with numpy so that the bench
configs (GiB-scale) build in seconds.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

BASE_SEED = 0x5EEDC0DE
GOLDEN = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)
HEX = np.frombuffer(b"0123456789abcdef", dtype=np.uint8)
ALNUM = np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789", dtype=np.uint8)

MiB = 1 << 20


def splitmix64(seed: int, n: int, start: int = 0) -> np.ndarray:
    """n outputs of splitmix64 seeded with `seed`, starting at output index `start`."""
    with np.errstate(over="ignore"):
        i = np.arange(start + 1, start + n + 1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + i * GOLDEN
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def mix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser as a hash of an id array."""
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) * GOLDEN + np.uint64(0x632BE59BD9B4E019)
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def hex16(x: np.ndarray) -> np.ndarray:
    """u64 array -> (n, 16) lowercase hex bytes; hex order == numeric order."""
    shifts = np.arange(60, -4, -4, dtype=np.uint64)
    nib = (x[:, None] >> shifts[None, :]) & np.uint64(0xF)
    return HEX[nib.astype(np.intp)]


def random_bytes(seed: int, n: int) -> np.ndarray:
    words = splitmix64(seed, (n + 7) // 8)
    return words.view(np.uint8)[:n]


def unique_sorted_u64(seed: int, n: int, universe: int = 0) -> np.ndarray:
    """n distinct sorted u64 draws (from [0, universe) when universe > 0)."""
    got = np.empty(0, dtype=np.uint64)
    start = 0
    while got.size < n:
        need = n - got.size
        draw = splitmix64(seed, need + need // 8 + 16, start)
        start += draw.size
        if universe:
            draw = draw % np.uint64(universe)
        got = np.unique(np.concatenate([got, draw]))
    if got.size > n:  # keep a deterministic subset: drop by hash rank
        h = mix64(got ^ np.uint64(seed & 0xFFFFFFFFFFFFFFFF))
        keep = np.sort(np.argsort(h, kind="stable")[:n])
        got = got[keep]
    return got


def assemble_run(keys: Sequence[np.ndarray] | np.ndarray, vals, is_put: np.ndarray) -> np.ndarray:
    """Serialise records into one v1 run (uint8 array).

    keys: (n, K) uint8 fixed-width, or (flat uint8, lengths) tuple for variable width.
    vals: (n, V) uint8 fixed-width (used only for Puts), or (flat, lengths) tuple.
    """
    if isinstance(keys, tuple):
        kflat, klen = keys
    else:
        n, kw = keys.shape
        kflat, klen = keys.reshape(-1), np.full(n, kw, dtype=np.int64)
    n = klen.size
    if isinstance(vals, tuple):
        vflat, vlen = vals
    else:
        vw = vals.shape[1] if vals.ndim == 2 else 0
        vflat, vlen = vals.reshape(-1), np.full(n, vw, dtype=np.int64)
    klen = klen.astype(np.int64)
    vlen = np.where(is_put, vlen.astype(np.int64), 0)
    sizes = np.where(is_put, 9 + klen + vlen, 5 + klen)
    offs = np.empty(n, dtype=np.int64)
    if n:
        offs[0] = 1
        np.cumsum(sizes[:-1], out=offs[1:])
        offs[1:] += 1
    total = 1 + int(sizes.sum())
    out = np.zeros(total, dtype=np.uint8)
    out[0] = 1
    out[offs] = np.where(is_put, 1, 2).astype(np.uint8)
    kl = klen.astype(">u4").view(np.uint8).reshape(n, 4)
    for j in range(4):
        out[offs + 1 + j] = kl[:, j]
    # keys
    kstart = np.zeros(n, dtype=np.int64)
    if n:
        np.cumsum(klen[:-1], out=kstart[1:])
    tk = int(klen.sum())
    if tk:
        dst = np.repeat(offs + 5 - kstart, klen) + np.arange(tk, dtype=np.int64)
        out[dst] = kflat[:tk]
    # values (puts only)
    pv = np.nonzero(is_put)[0]
    if pv.size:
        vo = offs[pv] + 5 + klen[pv]
        vl = vlen[pv].astype(">u4").view(np.uint8).reshape(pv.size, 4)
        for j in range(4):
            out[vo + j] = vl[:, j]
        if isinstance(vals, tuple):
            vstart_all = np.zeros(n, dtype=np.int64)
            if n:
                np.cumsum(vals[1][:-1].astype(np.int64), out=vstart_all[1:])
            src_start = vstart_all[pv]
        else:
            src_start = pv.astype(np.int64) * (vals.shape[1] if vals.ndim == 2 else 0)
        lens = vlen[pv]
        tv = int(lens.sum())
        if tv:
            rel = np.arange(tv, dtype=np.int64) - np.repeat(np.concatenate([[0], np.cumsum(lens)[:-1]]), lens)
            dst = np.repeat(vo + 4, lens) + rel
            src = np.repeat(src_start, lens) + rel
            out[dst] = vflat[src]
    return out


# ----------------------------------------------------------------------------------------
# config shapes (BASELINE.json "configs")

def hex_key_run(seed: int, n: int, vsize: int, universe: int = 0) -> np.ndarray:
    ids = unique_sorted_u64(seed, n, universe)
    keys = hex16(ids)
    vals = random_bytes(seed ^ 0xA5A5A5A5, n * vsize).reshape(n, vsize)
    return assemble_run(keys, vals, np.ones(n, dtype=bool))


def config1(seed: int = BASE_SEED, n_records: int = 11781):
    """2-way table-buffer compaction, 2 x ~1 MiB runs, 16 B hex keys over a 2^20 universe
    (so the runs overlap), 64 B values. SeqNo 1, 2."""
    return [(s + 1, [hex_key_run(seed + s, n_records, 64, universe=1 << 20).tobytes()]) for s in range(2)]


def config2(seed: int = BASE_SEED, n_streams: int = 64, n_records: int = 238821, vsize: int = 256,
            variant: str = "A"):
    """64-way L0->L1 compaction: n_streams x 1 run x n_records; 16 B hex keys, 256 B values.
    Variant A: keys uniform over 2^64 (no superseded records). Variant B: keys from a
    universe of n_streams*n_records ids (~37 % superseded at full size)."""
    universe = 0 if variant == "A" else n_streams * n_records
    return [(s + 1, [hex_key_run(seed + s, n_records, vsize, universe).tobytes()]) for s in range(n_streams)]


def l0_ids(seed: int, n_buffer: int, n_l0: int, run_records: int):
    """Key ids of a table-buffer compaction with a concatenated L0: (buffer id arrays, L0 id arrays).
    One universe of 2 x all records, so buffer records supersede some L0 records; the L0 runs hold
    consecutive slices of one sorted id set (ascending, disjoint key ranges, as build_runs' outputs)."""
    universe = 2 * (n_buffer + n_l0) * run_records
    l0 = unique_sorted_u64(seed, n_l0 * run_records, universe)
    buf = [unique_sorted_u64(seed + 1 + b, run_records, universe) for b in range(n_buffer)]
    return buf, [l0[i * run_records:(i + 1) * run_records] for i in range(n_l0)]


def config_l0(seed: int = BASE_SEED, n_buffer: int = 16, n_l0: int = 1024, run_records: int = 14925,
              vsize: int = 256):
    """Table-buffer compaction with L0 (table_buffer_compaction.rs:31-100): n_buffer buffer runs at
    SeqNo 1..n_buffer plus ONE stream at SeqNo 0 concatenating n_l0 ascending L0 runs; config 2's
    record shape (16 B hex keys, vsize B values; 14,925 records = one 4 MiB run)."""
    buf, l0 = l0_ids(seed, n_buffer, n_l0, run_records)

    def run(ids, tag):
        vals = random_bytes(seed ^ (0x3C3C + tag), ids.size * vsize).reshape(ids.size, vsize)
        return assemble_run(hex16(ids), vals, np.ones(ids.size, dtype=bool)).tobytes()

    streams = [(b + 1, [run(ids, b)]) for b, ids in enumerate(buf)]
    streams.append((0, [run(ids, 1000 + i) for i, ids in enumerate(l0)]))
    return streams


def alnum_keys(ids: np.ndarray, min_len: int = 8, max_len: int = 128):
    """Deterministic alnum key of each id (length min..max); returns (flat, lengths)."""
    h = mix64(ids)
    lens = (min_len + (h % np.uint64(max_len - min_len + 1))).astype(np.int64)
    total = int(lens.sum())
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    pos = np.arange(total, dtype=np.int64) - np.repeat(starts, lens)
    hid = np.repeat(ids.astype(np.uint64), lens)
    ch = mix64(hid * np.uint64(1315423911) + pos.astype(np.uint64))
    flat = ALNUM[(ch % np.uint64(62)).astype(np.intp)]
    return flat, lens


def var_key_run(seed: int, n: int, universe: int, vsize: int = 256, delete_frac: float = 0.10,
                min_len: int = 8, max_len: int = 128) -> np.ndarray:
    """Variable-length alnum keys (8-128 B) drawn from a shared id universe (so runs overlap),
    sorted bytewise, 10 % Deletes."""
    ids = unique_sorted_u64(seed, n, universe)
    flat, lens = alnum_keys(ids, min_len, max_len)
    # sort bytewise: fixed-width 'S' compare == lexicographic for NUL-free keys
    width = int(lens.max()) if lens.size else 1
    mat = np.zeros((n, width), dtype=np.uint8)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    rows = np.repeat(np.arange(n), lens)
    cols = np.arange(int(lens.sum())) - np.repeat(starts, lens)
    mat[rows, cols] = flat
    order = np.argsort(mat.view(f"S{width}").reshape(-1), kind="stable")
    sk = mat.view(f"S{width}").reshape(-1)[order]
    uniq = np.ones(n, dtype=bool)
    uniq[1:] = sk[1:] != sk[:-1]
    order = order[uniq]
    lens_s = lens[order]
    mat_s = mat[order]
    n2 = order.size
    flat_s = mat_s[np.repeat(np.arange(n2), lens_s), np.arange(int(lens_s.sum())) - np.repeat(
        np.concatenate([[0], np.cumsum(lens_s)[:-1]]), lens_s)]
    r = mix64(ids[order] ^ np.uint64(seed & 0xFFFFFFFF))
    is_put = (r % np.uint64(1000)) >= np.uint64(int(delete_frac * 1000))
    vals = random_bytes(seed ^ 0x5A5A5A5A, n2 * vsize).reshape(n2, vsize)
    return assemble_run((flat_s, lens_s), vals, is_put)


def config3(seed: int = BASE_SEED, n_streams: int = 256, run_bytes: int = 256 * MiB, vsize: int = 256):
    """256-way compaction, variable-length keys 8-128 B + 10 % tombstones. Each run holds
    about run_bytes of records (mean record ~333 B)."""
    n = max(1, run_bytes // 333)
    universe = n * n_streams * 2
    return [(s + 1, [var_key_run(seed + s, n, universe, vsize).tobytes()]) for s in range(n_streams)]


def wal_run(seed: int, n: int = 83, n_tables: int = 64, key_len: int = 32, vsize: int = 8) -> np.ndarray:
    """One WAL run: n records with keys "{table_id}." + zero-padded suffix (32 B), 8 B values."""
    r = splitmix64(seed, 2 * n + 8)
    tables = (r[:n] % np.uint64(n_tables)).astype(np.int64)
    suff = r[n:2 * n] % np.uint64(10 ** 12)
    keys = []
    for t, s in zip(tables.tolist(), suff.tolist()):
        p = f"{t}."
        keys.append((p + str(s).zfill(key_len - len(p))).encode())
    keys = sorted(set(keys))
    m = len(keys)
    kmat = np.frombuffer(b"".join(keys), dtype=np.uint8).reshape(m, key_len)
    vals = random_bytes(seed ^ 0x77, m * vsize).reshape(m, vsize)
    return assemble_run(kmat, vals, np.ones(m, dtype=bool))


def config5(seed: int = BASE_SEED, n_streams: int = 1_000_000, n_records: int = 83):
    """WAL -> table-buffer flush: many tiny WAL runs (83 x 49 B records = 4,068 B)."""
    return [(s + 1, [wal_run(seed + s, n_records).tobytes()]) for s in range(n_streams)]


def total_bytes(streams) -> int:
    return sum(len(r) for _, runs in streams for r in runs)
