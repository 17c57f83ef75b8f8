"""Synthetic BASELINE workloads built directly in HBM — shared by bench.py and
the full-size parity tests (tests/test_gpu_fullsize.py). Bench/test infrastructure: the product
path never imports this module. Every generator is deterministic in its seed.
"""
from __future__ import annotations

import numpy as np
import torch

from . import gen


def make_cfg2_on_device(device, seed, n_streams, n_records, vsize, variant="A"):
    """Each stream: one v1 run of n_records Put records with sorted unique 16 B hex keys and
    random values, built directly in HBM (keys from splitmix64 on the host, values from the
    device RNG)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    rec = 9 + 16 + vsize
    runs = []
    universe = 0 if variant == "A" else n_streams * n_records
    hdr = torch.tensor([1, 0, 0, 0, 16], dtype=torch.uint8, device=device)
    vl = torch.tensor(list(int(vsize).to_bytes(4, "big")), dtype=torch.uint8, device=device)
    for s in range(n_streams):
        ids = gen.unique_sorted_u64(seed + s, n_records, universe)
        keys = torch.from_numpy(np.ascontiguousarray(gen.hex16(ids))).to(device)
        run = torch.empty(1 + n_records * rec, dtype=torch.uint8, device=device)
        run[0] = 1
        body = run[1:].view(n_records, rec)
        body[:, 0:5] = hdr
        body[:, 5:21] = keys
        body[:, 21:25] = vl
        body[:, 25:] = torch.randint(0, 256, (n_records, vsize), dtype=torch.uint8, device=device, generator=g)
        runs.append(run)
    torch.cuda.synchronize(device)
    return runs


def _hex_run_on_device(device, ids, vsize, g):
    """One v1 run of Puts with 16 B hex keys of the sorted ids and device-RNG values, in HBM."""
    rec = 9 + 16 + vsize
    n = int(ids.size)
    run = torch.empty(1 + n * rec, dtype=torch.uint8, device=device)
    run[0] = 1
    body = run[1:].view(n, rec)
    body[:, 0:5] = torch.tensor([1, 0, 0, 0, 16], dtype=torch.uint8, device=device)
    body[:, 5:21] = torch.from_numpy(np.ascontiguousarray(gen.hex16(ids))).to(device)
    body[:, 21:25] = torch.tensor(list(int(vsize).to_bytes(4, "big")), dtype=torch.uint8, device=device)
    body[:, 25:] = torch.randint(0, 256, (n, vsize), dtype=torch.uint8, device=device, generator=g)
    return run


def make_l0_on_device(device, seed, n_buffer=16, n_l0=1024, run_records=14925, vsize=256):
    """gen.config_l0's shape built in HBM: (buffer runs, L0 member runs). Stream table: buffer run b
    at SeqNo b + 1, the L0 runs concatenated as one stream at SeqNo 0."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    buf, l0 = gen.l0_ids(seed, n_buffer, n_l0, run_records)
    bruns = [_hex_run_on_device(device, ids, vsize, g) for ids in buf]
    lruns = [_hex_run_on_device(device, ids, vsize, g) for ids in l0]
    torch.cuda.synchronize(device)
    return bruns, lruns


def make_cfg3_on_device(device, seed, n_streams, run_mib, vsize=256):
    """Config 3 (scaled): gen.config3's runs (variable-length sorted alnum keys, 10 % Deletes)
    built on the host, copied to HBM."""
    streams = gen.config3(seed=seed, n_streams=n_streams, run_bytes=run_mib << 20, vsize=vsize)
    runs = [torch.frombuffer(bytearray(r[1][0]), dtype=torch.uint8).to(device) for r in streams]
    torch.cuda.synchronize(device)
    return runs


def make_cfg3_full_on_device(device, seed, n_streams, run_mib, vsize=256, with_index=False):
    """Config 3 at BASELINE size, built in HBM: per stream ~run_mib MiB of records whose keys are
    an order-preserving 5-character base-62 rendering of a sorted unique id (ids drawn from a
    universe shared by all streams, so streams overlap and equal ids give equal keys; 62^5 =
    9.2e8 covers the 4.1e8-id universe of BASELINE's 256 x 256 MiB) plus a deterministic alnum
    tail, 8-128 B in all (BASELINE's 8-128 B, so keys shorter than the 16-byte
    prefix, zero-padded in the device key words, occur); 10 % Deletes; 256 B random values.
    with_index: also return each stream's (ids, record offsets) — key order is id order, so the
    full-size tests cut every stream into the same key ranges without parsing it."""
    n = (run_mib << 20) // 333
    universe = n * n_streams * 2
    assert universe <= 62 ** 5, "ids must fit the 5-character prefix"
    M = 0x7FFFFFFFFFFFFFFF

    def h(x):  # a 63-bit integer mix (deterministic, non-negative)
        x = (x * 0x5851F42D4C957F2D + 0x14057B7EF767814F) & M
        x = x ^ (x >> 29)
        x = (x * 0x2545F4914F6CDD1D) & M
        return x ^ (x >> 32)

    alnum = torch.tensor(list(b"0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz"), dtype=torch.int64,
                         device=device)
    pow62 = torch.tensor([62 ** (4 - i) for i in range(5)], dtype=torch.int64, device=device)
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    runs, index = [], []
    for s in range(n_streams):
        ids = torch.unique(torch.randint(0, universe, (n + n // 20,), generator=g, device=device))[:n]
        m = ids.numel()
        klen = 8 + h(ids) % 121
        is_put = h(ids ^ (seed + 7919 * s)) % 1000 >= 100
        size = 5 + klen + torch.where(is_put, 4 + vsize, 0)
        off = torch.cumsum(size, 0) - size + 1
        total = int(off[-1] + size[-1])
        buf = torch.empty(total, dtype=torch.uint8, device=device)
        buf[0] = 1
        buf[off] = torch.where(is_put, 1, 2).to(torch.uint8)
        for b in range(4):
            buf[off + 1 + b] = ((klen >> (8 * (3 - b))) & 0xFF).to(torch.uint8)
        kidx = torch.repeat_interleave(torch.arange(m, device=device), klen)
        kpos = torch.arange(kidx.numel(), device=device) - torch.repeat_interleave(torch.cumsum(klen, 0) - klen, klen)
        kid = ids[kidx]
        digit = torch.where(kpos < 5, (kid // pow62[kpos.clamp(max=4)]) % 62, h(kid * 131 + kpos) % 62)
        buf[off[kidx] + 5 + kpos] = alnum[digit].to(torch.uint8)
        del kidx, kpos, kid, digit
        pidx = torch.nonzero(is_put).squeeze(1)
        vo = off[pidx] + 5 + klen[pidx]
        for b in range(4):
            buf[vo + b] = (vsize >> (8 * (3 - b))) & 0xFF
        vpos = (vo + 4).unsqueeze(1) + torch.arange(vsize, device=device)
        buf[vpos.reshape(-1)] = torch.randint(0, 256, (pidx.numel() * vsize,), dtype=torch.uint8, device=device,
                                              generator=g)
        del vpos, pidx, vo
        runs.append(buf)
        if with_index:
            index.append((ids, off))
    torch.cuda.synchronize(device)
    return (runs, index) if with_index else runs


def make_cfg5_on_device(device, seed, n_streams, n_records=83, n_tables=64):
    """Config 5: n_streams WAL runs of n_records Puts, key "{t}." + zero-filled decimal suffix
    (32 B, gen.wal_run's format), 8 B values, each run sorted bytewise; one HBM tensor."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    N = n_streams * n_records
    t = torch.randint(0, n_tables, (N,), device=device, generator=g)
    suf = torch.randint(0, 10 ** 12, (N,), device=device, generator=g, dtype=torch.int64)
    keys = torch.full((N, 32), ord("0"), dtype=torch.int64, device=device)
    two = t < 10
    keys[:, 0] = torch.where(two, t, t // 10) + ord("0")
    keys[:, 1] = torch.where(two, torch.full_like(t, ord(".")), t % 10 + ord("0"))
    keys[:, 2] = torch.where(two, torch.full_like(t, ord("0")), torch.full_like(t, ord(".")))
    x = suf.clone()
    for i in range(31, 19, -1):
        keys[:, i] = x % 10 + ord("0")
        x //= 10
    # bytewise order inside each run: stable LSD sorts over the four big-endian 8-byte words
    w = (keys.view(N, 4, 8) << torch.tensor([56, 48, 40, 32, 24, 16, 8, 0], device=device)).sum(dim=2)
    w = w.view(n_streams, n_records, 4)
    order = torch.arange(n_records, device=device).expand(n_streams, n_records).contiguous()
    for q in (3, 2, 1, 0):
        vals = torch.gather(w[:, :, q], 1, order)
        _, o = torch.sort(vals, dim=1, stable=True)
        order = torch.gather(order, 1, o)
    rows = torch.arange(n_streams, device=device).unsqueeze(1) * n_records
    keys = keys.to(torch.uint8)[(rows + order).reshape(-1)]
    rec = torch.empty((N, 49), dtype=torch.uint8, device=device)
    rec[:, 0:5] = torch.tensor([1, 0, 0, 0, 32], dtype=torch.uint8, device=device)
    rec[:, 5:37] = keys
    rec[:, 37:41] = torch.tensor([0, 0, 0, 8], dtype=torch.uint8, device=device)
    rec[:, 41:49] = torch.randint(0, 256, (N, 8), dtype=torch.uint8, device=device, generator=g)
    run_len = 1 + n_records * 49
    buf = torch.empty((n_streams, run_len), dtype=torch.uint8, device=device)
    buf[:, 0] = 1
    buf[:, 1:] = rec.view(n_streams, n_records * 49)
    del rec, keys, w, order, t, suf, x
    torch.cuda.synchronize(device)
    return buf
