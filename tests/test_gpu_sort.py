"""GPU parity of the record sort (skv_sort.hip): merges of more than TILE_TARGET / 2 = 1536
streams (config 5's 10^6 WAL runs) sort the records by (key, record index) into one list before
the level-0 merge stage. Same bar as test_gpu_parity: output bytes, StatsV1, dropped tables and
the first error, bit-exact against the CPU restatement (oracle/).

SKV_SORT=1 forces the sort at any fan-in, so the reference-derived fixtures and the random
domain run through it as well."""
import json
import os
import random

import pytest

from skv import _abi, gen
from skv import format as fmt
from skv.api import Compactor

from test_gpu_parity import _case, _diff, _run_both
from knobs import knob, knob_get  # noqa: E402

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = json.load(open(os.path.join(GOLDEN, "compact_cases.json")))
MiB = 1 << 20


@pytest.fixture(scope="module")
def dev():
    torch = pytest.importorskip("torch")
    torch.cuda.init()
    c = Compactor(0, profiling=True)
    yield c
    c.close()


@pytest.fixture
def forced_sort(monkeypatch):
    knob("SKV_SORT", "1")
    knob("SKV_FUSED", "0")


def _check(dev, streams, max_size, flags, expect_sorted=True):
    exp, got = _run_both(dev, streams, max_size, flags)
    assert exp == got, _diff(exp, got)
    if expect_sorted and got[0] == "ok" and got[1]:
        assert dev.timings()["sorted"] == 1, "the record sort did not run"
    return got


def test_forced_sort_golden_fixtures(dev, forced_sort):
    bad = []
    for case in CASES:
        streams = [(s, [bytes.fromhex(r) for r in runs]) for s, runs in case["streams"]]
        exp, got = _run_both(dev, streams, case["max"], case["flags"])
        if exp != got:
            bad.append((case["name"], _diff(exp, got)))
    assert not bad, bad[:5]


def test_forced_sort_random_cases(dev, forced_sort):
    bad, n = [], 0
    for seed in range(400):
        streams, max_size, flags = _case(seed)
        exp, got = _run_both(dev, streams, max_size, flags)
        if got[0] == "err" and got[1] == _abi.SKV_E_UNSUPPORTED:
            continue
        n += 1
        if exp != got:
            bad.append((seed, _diff(exp, got)))
    assert n > 200
    assert not bad, f"{len(bad)} mismatches, first: {bad[:5]}"


@pytest.mark.parametrize("name,streams,max_size,flags", [
    ("cfg2B", lambda: gen.config2(n_streams=16, n_records=3000, vsize=40, variant="B"), 256 * 1024, 0),
    ("cfg3_var_keys", lambda: gen.config3(n_streams=24, run_bytes=96 * 1024, vsize=32), 128 * 1024, 0),
    ("cfg3_drop", lambda: gen.config3(n_streams=24, run_bytes=96 * 1024, vsize=32), 128 * 1024, 1),
    ("cfg5_wal", lambda: gen.config5(n_streams=300), 4 * MiB, 2),
])
def test_forced_sort_generated(dev, forced_sort, name, streams, max_size, flags):
    _check(dev, streams(), max_size, flags)


def test_fan_in_2000_wal_runs(dev):
    """Config-5 shape past the splitter merge's fan-in: 2000 WAL runs of 83 records (32-byte
    "{table}.{suffix}" keys whose first 16 bytes mostly agree, so every bucket sorts on the bytes
    after its splitters' common prefix)."""
    _check(dev, gen.config5(n_streams=2000), 4 * MiB, _abi.SKV_SPLIT_BY_TABLE)


def test_fan_in_wal_runs_with_same_size_deletes(dev):
    """Fixed-stride WAL runs of one format take one meta for every sorted record (k_sort_store's
    const_meta) -- unless a record is a Delete of the runs' record size (key of S - 5 bytes), which
    the fixed-stride parse accepts: then the meta of each record is gathered. Both outcomes equal the
    oracle's, with and without the Delete filter."""
    streams = gen.config5(n_streams=1700)
    S = len(streams[0][1][0]) // 83  # 49-byte Puts: 1 + 4 + 32 + 4 + 8
    _check(dev, streams, 4 * MiB, _abi.SKV_SPLIT_BY_TABLE)
    r = random.Random(17)
    for i in r.sample(range(len(streams)), 40):
        seq, (run,) = streams[i]
        recs = [run[1 + j * S:1 + (j + 1) * S] for j in range(83)]
        j = r.randrange(83)
        key = recs[j][5:37] + b"~" * (S - 5 - 32)  # sorts right after its Put's key, before the next
        if j + 1 < 83 and key >= recs[j + 1][5:5 + 32]:
            continue
        dele = fmt.encode_record(fmt.delete(key.decode()))
        assert len(dele) == S
        recs[j + 1:j + 1] = [dele]
        streams[i] = (seq, [run[:1] + b"".join(recs[:83]) + b"".join(recs[83:])])
    for flags in (_abi.SKV_SPLIT_BY_TABLE, _abi.SKV_SPLIT_BY_TABLE | _abi.SKV_DROP_TOMBSTONES):
        _check(dev, streams, 4 * MiB, flags)


def test_fan_in_1600_overlapping_streams(dev):
    """1600 streams over a shared key universe: superseded records across streams (newest wins)."""
    streams = gen.config2(n_streams=1600, n_records=60, vsize=12, variant="B")
    _check(dev, streams, 64 * 1024, 0)


def test_fan_in_var_keys_with_tombstones(dev):
    streams = gen.config3(n_streams=1700, run_bytes=6000, vsize=16)
    _check(dev, streams, 256 * 1024, 0)
    _check(dev, streams, 256 * 1024, _abi.SKV_DROP_TOMBSTONES)


def test_fan_in_equal_key_flood(dev):
    """3000 streams holding the same few keys: one bucket far above SORT_CAP (the global-memory
    bucket sort), the newest seq_no wins each key."""
    r = random.Random(5)
    streams = []
    for s in range(3000):
        keys = sorted({f"k{r.randrange(4)}" for _ in range(3)} | {f"u{s:05d}"})
        ops = [fmt.put(k, s.to_bytes(4, "big")) if r.random() < 0.8 else fmt.delete(k) for k in keys]
        streams.append((s * 7 - 9000, [fmt.encode_run(ops)]))
    _check(dev, streams, 1 << 14, 0)
    _check(dev, streams, 1 << 14, _abi.SKV_DROP_TOMBSTONES)


def test_fan_in_long_shared_prefixes(dev):
    """Keys of 40-90 bytes sharing a 35-byte prefix, plus keys that are prefixes of others."""
    r = random.Random(9)
    base = "tenant-0001/namespace/partition-000/"
    streams = []
    for s in range(1800):
        ks = set()
        for _ in range(r.randint(1, 8)):
            tail = "".join(r.choice("ab") for _ in range(r.randint(0, 50)))
            ks.add((base + tail).encode())
        ops = [fmt.put(k, bytes([s & 255])) for k in sorted(ks)]
        streams.append((s + 1, [fmt.encode_run(ops)]))
    _check(dev, streams, 1 << 16, 0)


def test_fan_in_tie_runs_past_the_first_word(dev):
    """The bucket sort orders 8-byte words first: keys whose words tie and which differ only
    later (runs of 2-40 equal words, some past SORT_TIE_MAX -> the global-memory bucket sort),
    duplicates across streams, and keys that are prefixes of others inside one tie run."""
    r = random.Random(21)
    streams = []
    for s in range(1700):
        ks = set()
        for _ in range(r.randint(1, 6)):
            grp = r.randrange(60)
            head = f"g{grp:04d}-" + "x" * (grp % 9)
            ks.add((head + "".join(r.choice("pq") for _ in range(r.randint(0, 6 + grp % 5)))).encode())
        ops = [fmt.put(k, s.to_bytes(2, "big")) if r.random() < 0.9 else fmt.delete(k) for k in sorted(ks)]
        streams.append((3 * s + 1, [fmt.encode_run(ops)]))
    _check(dev, streams, 1 << 15, 0)
    _check(dev, streams, 1 << 15, _abi.SKV_DROP_TOMBSTONES)


@pytest.mark.parametrize("nt,two,gmax", [("4", "1", "16"), ("16", "1", "16"), ("16", "1", "0"), ("4", "0", "16")])
def test_bucket_levels_at_small_sizes(dev, monkeypatch, nt, two, gmax):
    """SKV_SB_NT caps the bucket search's LDS level at nt entries, so its group level runs at test
    sizes: with SKV_SORT_TWO_PASS=1 the two-pass bucketing (k_sort_pass_a: super-buckets in LDS;
    k_sort_pass_b: each chunk's groups' windows from the super-bucket prefix in LDS, or from the
    global table when a chunk spans more than SKV_SB_GMAX groups), with 0 the one-pass search
    through the global discriminators. WAL keys, long shared prefixes, tie runs past the sort word, an equal-key flood
    and variable keys with tombstones, all against the oracle."""
    knob("SKV_SB_NT", nt)
    knob("SKV_SORT_TWO_PASS", two)
    knob("SKV_SB_GMAX", gmax)
    _check(dev, gen.config5(n_streams=2000), 4 * MiB, _abi.SKV_SPLIT_BY_TABLE)
    r = random.Random(9)
    base = "tenant-0001/namespace/partition-000/"
    streams = []
    for s in range(1800):
        ks = {(base + "".join(r.choice("ab") for _ in range(r.randint(0, 50)))).encode()
              for _ in range(r.randint(1, 8))}
        streams.append((s + 1, [fmt.encode_run([fmt.put(k, bytes([s & 255])) for k in sorted(ks)])]))
    _check(dev, streams, 1 << 16, 0)
    r = random.Random(21)
    streams = []
    for s in range(1700):
        ks = set()
        for _ in range(r.randint(1, 6)):
            grp = r.randrange(60)
            head = f"g{grp:04d}-" + "x" * (grp % 9)
            ks.add((head + "".join(r.choice("pq") for _ in range(r.randint(0, 6 + grp % 5)))).encode())
        ops = [fmt.put(k, s.to_bytes(2, "big")) if r.random() < 0.9 else fmt.delete(k) for k in sorted(ks)]
        streams.append((3 * s + 1, [fmt.encode_run(ops)]))
    _check(dev, streams, 1 << 15, _abi.SKV_DROP_TOMBSTONES)
    r = random.Random(5)
    streams = []
    for s in range(3000):
        keys = sorted({f"k{r.randrange(4)}" for _ in range(3)} | {f"u{s:05d}"})
        ops = [fmt.put(k, s.to_bytes(4, "big")) if r.random() < 0.8 else fmt.delete(k) for k in keys]
        streams.append((s * 7 - 9000, [fmt.encode_run(ops)]))
    _check(dev, streams, 1 << 14, 0)
    _check(dev, gen.config3(n_streams=1700, run_bytes=6000, vsize=16), 256 * 1024, _abi.SKV_DROP_TOMBSTONES)


@pytest.mark.parametrize("order", ["ascending", "descending", "shuffled"])
def test_wide_one_run_streams_by_caller_order(dev, order):
    """70,000 one-run streams (past build_job's 65,536-stream threshold for host-thread blocks):
    in a strict seq_no order every block writes its tables in pass 1 and the run table is built on
    the device (k_run_info, reversed for an ascending caller order); shuffled, pass 2 and the host
    run table do it. Same output and stats as the oracle either way."""
    r = random.Random(41)
    n = 70_000
    streams = []
    for s in range(n):
        keys = sorted({f"{r.randrange(8)}.{r.randrange(10 ** 9):09d}" for _ in range(2)})
        ops = [fmt.put(k, bytes([s & 255, 7])) if r.random() < 0.9 else fmt.delete(k) for k in keys]
        streams.append((s + 1, [fmt.encode_run(ops)]))
    if order == "descending":
        streams.reverse()
    elif order == "shuffled":
        r.shuffle(streams)
    _check(dev, streams, 1 << 20, _abi.SKV_SPLIT_BY_TABLE)
    _check(dev, streams, 1 << 20, 0)


def test_fan_in_errors_surface_like_the_reference(dev):
    """A corrupt or unsorted stream among 1600: the error is resolved before the sort."""
    r = random.Random(3)
    streams = []
    for s in range(1600):
        ops = [fmt.put(f"{r.randrange(10**6):07d}", b"v") for _ in range(5)]
        ops = sorted({o[1]: o for o in ops}.values(), key=lambda o: o[1])
        streams.append((s + 1, [fmt.encode_run(ops)]))
    bad = bytearray(streams[777][1][0])
    bad[0] = 3  # unsupported version
    streams[777] = (streams[777][0], [bytes(bad)])
    exp, got = _run_both(dev, streams, 4 * MiB, 0)
    assert exp == got, _diff(exp, got)


# ---- the level-0 merge's key-fingerprint shortcut (skv_kernels.hip elem_less_fp) -----------------

def _prefix_keys_streams(n_streams=12, per=300, seed=11):
    """Keys sharing their first 16 bytes, same length, distinct tails, spread over many streams:
    under SKV_FP_TEST=1 (all fingerprints 0) the merge rounds take them as equal and misorder
    them, which the exact adjacency check must catch."""
    r = random.Random(seed)
    streams = []
    for s in range(n_streams):
        ks = sorted({f"shared-prefix-16/{r.randrange(10**6):06d}" for _ in range(per)})
        ops = [fmt.put(k, bytes([s])) for k in ks]
        streams.append((s + 1, [fmt.encode_run(ops)]))
    return streams


def test_fp_shortcut_collisions_are_caught(dev, monkeypatch):
    knob("SKV_FUSED", "0")
    knob("SKV_FP_TEST", "1")
    streams = _prefix_keys_streams()
    _check(dev, streams, 1 << 16, 0, expect_sorted=False)
    assert dev.timings()["fp_rerun"] == 1, "forced collisions were not detected"
    _check(dev, streams, 1 << 16, _abi.SKV_DROP_TOMBSTONES, expect_sorted=False)


def test_fp_collisions_caught_by_the_gather(dev, monkeypatch):
    """Every forced collision pairs a survivor with the one record dropped after it (two keys per
    16-byte prefix, in different streams): only k_gather's in-gather verify (TileOut::m_dup) sees
    them. With SKV_FP_GATHER=0 the same pairs go to k_fp_verify. Both detect and rerun exactly."""
    knob("SKV_FUSED", "0")
    r = random.Random(21)
    prefixes = sorted({f"p{r.randrange(10**12):015d}" for _ in range(3000)})
    a = fmt.encode_run([fmt.put(p + "aaaa", b"A") for p in prefixes])
    b = fmt.encode_run([fmt.put(p + "bbbb", b"B") for p in prefixes[::2]])
    c = fmt.encode_run([fmt.put(p + "aaaa", b"C") for p in prefixes[1::2]])  # real duplicates, other prefixes
    streams = [(3, [a]), (2, [b]), (1, [c])]
    for gather in ("1", "0"):
        knob("SKV_FP_GATHER", gather)
        knob("SKV_FP_TEST", "1")
        _check(dev, streams, 1 << 16, 0, expect_sorted=False)
        assert dev.timings()["fp_rerun"] == 1, f"SKV_FP_GATHER={gather}: forced collisions not detected"
        knob("SKV_FP_TEST", "0")
        _check(dev, streams, 1 << 16, 0, expect_sorted=False)
        assert dev.timings()["fp_rerun"] == 0


def test_fp_shortcut_no_rerun_on_real_fingerprints(dev, monkeypatch):
    knob("SKV_FUSED", "0")
    for streams, mx, fl in ((_prefix_keys_streams(), 1 << 16, 0),
                            (gen.config3(n_streams=32, run_bytes=64 * 1024, vsize=16), 1 << 18, 0),
                            (gen.config3(n_streams=32, run_bytes=64 * 1024, vsize=16), 1 << 18, 1),
                            (gen.config5(n_streams=64), 4 * MiB, 2)):
        _check(dev, streams, mx, fl, expect_sorted=False)
        assert dev.timings()["fp_rerun"] == 0


def test_fp_shortcut_wal_collisions(dev, monkeypatch):
    """WAL split after a merge whose fingerprints all collide (config-5 keys: one 16-byte prefix
    per table): the WAL stage must see the rerun's exact merge."""
    knob("SKV_FP_TEST", "1")
    _check(dev, gen.config5(n_streams=40), 4 * MiB, _abi.SKV_SPLIT_BY_TABLE, expect_sorted=False)
    assert dev.timings()["fp_rerun"] == 1
