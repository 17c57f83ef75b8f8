"""GPU parity of the fused stride path (skv_stride.hip) against the oracle, bit-exact.

The fused path is taken when every run is fixed-stride with one record size S >= 32 and one key
length K <= 16 (BASELINE configs 1, 2, 4). These tests pin:
  - that it is the path taken (skv_timings.path == SKV_PATH_FUSED) on such shapes;
  - output bytes + StatsV1 equal to the oracle over key/value widths, stream counts, duplicate
    densities, run-size limits (arithmetic greedy split, runs.rs:211-238, incl. max < S + 1 and
    max 0/1) and L0-style multi-member streams;
  - that everything the run's first record did not promise (Deletes of the same size, a bad
    marker, a key decrease, splitter skew above FX_CAP) is caught on the device, rejected with
    its reason bit, and rerun on the exact path with the reference's outcome.
"""
import os
import random

import numpy as np
import pytest

from skv import _abi, gen
from skv import format as fmt
from skv.api import Compactor

import pyoracle
from test_gpu_parity import _diff, _run_both
from knobs import knob, knob_get  # noqa: E402

pytestmark = pytest.mark.gpu
KiB, MiB = 1 << 10, 1 << 20
FXR_RECORD, FXR_OVERSIZE, FXR_SPLIT, FXR_ORDER, FXR_SAMPLE = 1, 2, 4, 8, 16


@pytest.fixture(scope="module")
def dev():
    torch = pytest.importorskip("torch")
    torch.cuda.init()
    c = Compactor(0, profiling=True)
    yield c
    c.close()


def _keys(seed, n, K, universe=0, alphabet=b"0123456789abcdef"):
    """n sorted distinct K-byte keys over `alphabet` (lexicographic order == id order)."""
    ids = gen.unique_sorted_u64(seed, n, universe or len(alphabet) ** min(K, 15))
    digits = np.empty((n, K), dtype=np.uint8)
    x = ids.copy()
    base = np.uint64(len(alphabet))
    table = np.frombuffer(alphabet, dtype=np.uint8)
    for c in range(K - 1, -1, -1):
        digits[:, c] = table[(x % base).astype(np.int64)]
        x //= base
    return digits


def _run(seed, n, K, V, universe=0, alphabet=b"0123456789abcdef"):
    keys = _keys(seed, n, K, universe, alphabet)
    vals = gen.random_bytes(seed ^ 0x5A5A, n * V).reshape(n, V)
    return gen.assemble_run(keys, vals, np.ones(n, dtype=bool)).tobytes()


def _check(dev, streams, max_size, flags=0, fused=True):
    exp, got = _run_both(dev, streams, max_size, flags)
    assert exp == got, _diff(exp, got)
    t = dev.timings()
    if fused:
        assert t["path"] == _abi.PATH_FUSED, (t["path"], t["fused_reject"])
    return t


@pytest.mark.parametrize("K,V,k,n,universe,max_size", [
    (16, 256, 64, 700, 0, 4 * MiB),          # config-2 shape, scaled
    (16, 256, 64, 700, 64 * 700, 4 * MiB),   # config-2B duplicates across streams
    (16, 64, 2, 11781, 1 << 20, 4 * MiB),    # config-1 shape
    (16, 7, 9, 3000, 0, 64 * KiB),           # S = 32, the smallest fused record
    (8, 40, 5, 5000, 30000, 1000),           # short keys, many small output runs
    (1, 40, 3, 16, 16, 100),                 # 1-byte keys, every stream holds the same 16 keys
    (0, 31, 4, 1, 0, 4 * MiB),               # empty keys: one survivor (the newest)
    (13, 300, 1, 9000, 0, 64 * KiB),         # one stream: no merge rounds
    (16, 100, 37, 900, 37 * 300, 2 * KiB),   # odd stream count, heavy duplicates
    (16, 200, 200, 150, 0, 256 * KiB),       # 200-way
])
def test_fused_shapes(dev, K, V, k, n, universe, max_size):
    streams = [(s + 1, [_run(100 * s + K, n, K, V, universe)]) for s in range(k)]
    _check(dev, streams, max_size)


@pytest.mark.parametrize("max_size", [0, 1, 40, 41, 80, 81, 82, 121, 4000, 1 << 62])
def test_fused_run_size_limits(dev, max_size):
    """S = 40: max < S + 1 gives one record per run (a record alone over max still forms a run,
    runs.rs:219); the version byte counts toward the size (runs.rs:241-246)."""
    streams = [(s + 1, [_run(s, 300, 16, 15)]) for s in range(6)]
    _check(dev, streams, max_size)


def test_fused_l0_concatenation(dev):
    """buffer runs + an L0-style stream of many fixed-stride members at SeqNo 0
    (table_buffer_compaction.rs:67-100): members are located per record by binary search."""
    l0 = []
    for i in range(30):
        keys = _keys(1000 + i, 200, 16, universe=10 ** 6)
        keys[:, 0] = ord("a") + i // 10
        keys[:, 1] = ord("0") + i % 10
        vals = gen.random_bytes(i, 200 * 50).reshape(200, 50)
        l0.append(gen.assemble_run(keys, vals, np.ones(200, dtype=bool)).tobytes())
    bufs = []
    for s in range(1, 9):
        keys = _keys(s, 1500, 16, universe=10 ** 6)
        keys[:, 0] = ord("a") + s % 3
        order = np.lexsort(keys.T[::-1])
        keys = np.unique(keys[order], axis=0)
        vals = gen.random_bytes(s, keys.shape[0] * 50).reshape(-1, 50)
        bufs.append((s, [gen.assemble_run(keys, vals, np.ones(keys.shape[0], dtype=bool)).tobytes()]))
    _check(dev, bufs + [(0, l0)], 32 * KiB)


def test_fused_utf8_keys(dev):
    """Multi-byte UTF-8 keys take the full from_utf8 check (runs.rs:585-591); an invalid
    sequence falls back and reports the reference's error."""
    rng = random.Random(4)
    words = sorted({"".join(rng.choice("aé€z") for _ in range(5)) for _ in range(4000)})
    words = [w for w in words if len(w.encode()) <= 16]
    words = [w.encode().ljust(16, b"_") for w in words]
    words = sorted(set(words))
    ops = [(True, w, b"v" * 20) for w in words]
    run = fmt.encode_run(ops)
    other = fmt.encode_run([(True, w, b"o" * 20) for w in words[::3]])
    _check(dev, [(1, [run]), (2, [other])], 16 * KiB)
    bad = bytearray(run)
    assert len(words) > 700
    bad[1 + 45 * 700 + 5 + 3] = 0xFF  # a key byte of record 700
    _check(dev, [(1, [bytes(bad)]), (2, [other])], 16 * KiB, fused=False)
    assert dev.timings()["fused_reject"] & FXR_RECORD


def test_fused_rejects_fall_back(dev):
    """Inputs that look fixed-stride from their first record but are not, each rejected on the
    device with its reason and rerun on the exact path."""
    base = [(s + 1, [_run(s, 2000, 16, 30)]) for s in range(8)]
    S = 9 + 16 + 30

    def with_run(i, data):
        out = list(base)
        out[i] = (out[i][0], [data])
        return out

    # a Delete of the same size (5 + 50 == 9 + 16 + 30): decodes fine, not a Put
    ops = [(True, b"%016d" % i, b"x" * 30) for i in range(0, 600, 2)]
    ops += [(False, b"%016d" % i + b"d" * 34, None) for i in range(1, 600, 2)]
    ops.sort(key=lambda o: o[1])
    cases = [([(1, [fmt.encode_run(ops)]), (2, [_run(9, 100, 16, 30)])], FXR_RECORD)]
    # a bad marker deep inside a run
    r = bytearray(base[3][1][0])
    r[1 + S * 1234] = 7
    cases.append((with_run(3, bytes(r)), FXR_RECORD))
    # a key decrease inside a run (the tile's neighbour check or the splitters)
    keys = _keys(77, 2000, 16)
    keys[[800, 801]] = keys[[801, 800]]
    vals = gen.random_bytes(5, 2000 * 30).reshape(2000, 30)
    cases.append((with_run(5, gen.assemble_run(keys, vals, np.ones(2000, dtype=bool)).tobytes()),
                  FXR_ORDER | FXR_SAMPLE | FXR_SPLIT))
    for streams, why in cases:
        _check(dev, streams, 8 * KiB, fused=False)
        t = dev.timings()
        assert t["path"] != _abi.PATH_FUSED and t["fused_reject"] & why, (t["path"], t["fused_reject"])


def test_fused_oversized_tile_reruns(dev):
    """5,000 copies of one key across streams land in one tile (> FX_CAP): rejected and rerun
    on the exact path (tile_big), same bytes."""
    streams = []
    for s in range(50):
        keys = np.frombuffer(b"k" * 16, dtype=np.uint8).reshape(1, 16).repeat(100, axis=0)
        vals = gen.random_bytes(s, 100 * 20).reshape(100, 20)
        streams.append((s + 1, [gen.assemble_run(keys, vals, np.ones(100, dtype=bool)).tobytes()]))
    _check(dev, streams, 4 * MiB, fused=False)
    assert dev.timings()["fused_reject"] & FXR_OVERSIZE


def test_fused_matches_unfused(dev):
    """Same bytes with the fused path disabled (SKV_FUSED=0 selects the fixed-stride record
    pipeline): the two device paths agree on a config-2B-shaped input."""
    streams = gen.config2(n_streams=64, n_records=2500, vsize=256, variant="B")
    a = dev.compact(streams, 4 * MiB, 0)
    assert dev.timings()["path"] == _abi.PATH_FUSED
    knob("SKV_FUSED", "0")
    try:
        b = dev.compact(streams, 4 * MiB, 0)
        assert dev.timings()["path"] == _abi.PATH_FIXED
    finally:
        knob("SKV_FUSED", None)
    assert [(x.data, x.stats.min_key, x.stats.max_key) for x in a] == \
        [(y.data, y.stats.min_key, y.stats.max_key) for y in b]


def test_fused_random_shapes(dev):
    """Random fused-eligible shapes: stream counts, widths, duplicate density, limits."""
    r = random.Random(1234)
    bad = []
    for trial in range(40):
        K = r.choice([2, 5, 8, 11, 16])
        V = r.randint(max(0, 32 - 9 - K), 120)
        k = r.choice([1, 2, 3, 7, 16, 64, 130])
        n = r.randint(1, 3000)
        uni = r.choice([0, k * n, max(1, n // 2)])
        if K <= 3:
            uni = min(uni or 16 ** K, 16 ** K)
        if uni:
            n = min(n, uni)  # n distinct keys need a universe of at least n
        max_size = r.choice([0, 9 + K + V, 2 * (9 + K + V) + 1, 5000, 64 * KiB, 4 * MiB])
        streams = [(r.randrange(-10**12, 10**12) * 1000 + s, [_run(trial * 1000 + s, n, K, V, uni)]) for s in range(k)]
        exp, got = _run_both(dev, streams, max_size, 0)
        path = dev.timings()["path"]
        if exp != got or path != _abi.PATH_FUSED:
            bad.append((trial, K, V, k, n, path, _diff(exp, got) if exp != got else "path"))
    assert not bad, bad[:5]


def test_fused_key_decrease_positions(dev):
    """A key decrease at many positions of one stream (run start and end, sample spacings, random
    places, so some land on tile edges): every one is caught on the device by the sample check, a
    tile's neighbour check or the tile-edge check against the previous record (whose key the
    bounds search carries, k_fx_bounds), and the exact path reproduces the reference's outcome."""
    n, K, V = 3000, 16, 30
    base = [(s + 1, [_run(500 + s, n, K, V)]) for s in range(16)]
    r = random.Random(99)
    positions = [0, 1, 5, 6, 7, n // 2, n - 2] + r.sample(range(n - 1), 9)
    bad = []
    for p in positions:
        keys = _keys(505, n, K)
        keys[[p, p + 1]] = keys[[p + 1, p]]
        vals = gen.random_bytes(505 ^ 0x5A5A, n * V).reshape(n, V)
        streams = list(base)
        streams[5] = (6, [gen.assemble_run(keys, vals, np.ones(n, dtype=bool)).tobytes()])
        exp, got = _run_both(dev, streams, 64 * KiB, 0)
        t = dev.timings()
        if exp != got or t["path"] == _abi.PATH_FUSED or not t["fused_reject"] & (FXR_ORDER | FXR_SAMPLE | FXR_SPLIT):
            bad.append((p, t["path"], t["fused_reject"], exp == got))
    assert not bad, bad


@pytest.mark.parametrize("slots", ["1", "2", "5"])
def test_fused_short_tail_tiles(dev, slots):
    """The last generation of tiles at half size (splitter t at sorted sample t*m up to T1, then
    T1*m + (t - T1)*m/2): forced on small inputs by pretending only `slots` tiles fit the GPU at
    once; same bytes as the oracle, and the fused path is still the one taken."""
    knob("SKV_FX_TAIL_SLOTS", slots)
    try:
        r = random.Random(int(slots))
        for trial in range(6):
            k = r.choice([2, 7, 16, 64])
            n = r.randint(2000, 6000)
            uni = r.choice([0, k * n // 2])
            streams = [(s + 1, [_run(7000 + 100 * trial + s, n, 16, 40, uni)]) for s in range(k)]
            _check(dev, streams, r.choice([4 * MiB, 5000, 64 * KiB]))
    finally:
        knob("SKV_FX_TAIL_SLOTS", None)
