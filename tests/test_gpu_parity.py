"""GPU parity: libskv.so (HIP, gfx950) against the CPU restatement (oracle/) and the golden
fixtures — bit-exact output bytes, StatsV1 and the first error (kind + reference text).

Run on the MI355X box with `pytest -m gpu`. Everything here calls through the C ABI.
"""
import hashlib
import json
import os
import random

import pytest

from skv import _abi, gen
from skv import format as fmt
from skv.api import Compactor

import pyoracle
from test_oracle_vs_pyref import _case
from knobs import knob, knob_get  # noqa: E402

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = json.load(open(os.path.join(GOLDEN, "compact_cases.json")))
KiB, MiB = 1 << 10, 1 << 20


@pytest.fixture(scope="module")
def dev():
    # torch bundles its own HIP runtime under the same SONAME; initialise it first so that
    # libskv.so binds to that one runtime instead of loading a second copy.
    torch = pytest.importorskip("torch")
    torch.cuda.init()
    c = Compactor(0, profiling=True)
    yield c
    c.close()


def _norm(runs):
    return [(r.data, r.stats.min_key, r.stats.max_key, r.stats.size_bytes, r.stats.put_count,
             r.stats.delete_count, r.table_id) for r in runs]


def _run_both(dev, streams, max_size, flags):
    """(oracle outcome, device outcome): ("ok", runs, dropped_tables) or ("err", code, text)."""
    try:
        runs, info = pyoracle.compact(streams, max_size, flags, with_result=True)
        exp = ("ok", _norm(runs), info["dropped_tables"])
    except _abi.RunError as e:
        exp = ("err", e.code, e.message)
    try:
        runs, info = dev.compact(streams, max_size, flags, with_info=True)
        got = ("ok", _norm(runs), info["dropped_tables"])
    except _abi.RunError as e:
        got = ("err", e.code, e.message)
    return exp, got


def _diff(exp, got):
    if exp[0] != got[0] or exp[0] == "err":
        return f"expected {exp[:3] if exp[0] == 'err' else 'ok'} got {got[:3] if got[0] == 'err' else 'ok'}"
    a, b = exp[1], got[1]
    if exp[2] != got[2]:
        return f"dropped tables {exp[2]} vs {got[2]}"
    if len(a) != len(b):
        return f"run count {len(a)} vs {len(b)}"
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            j = next((q for q in range(min(len(x[0]), len(y[0]))) if x[0][q] != y[0][q]), None)
            return f"run {i}: stats {x[1:]} vs {y[1:]}; first byte diff at {j}, lens {len(x[0])} {len(y[0])}"
    return "?"


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_golden_fixture(dev, case):
    streams = [(s, [bytes.fromhex(r) for r in runs]) for s, runs in case["streams"]]
    exp = case["expect"]
    if "error_code" in exp:
        with pytest.raises(_abi.RunError) as ei:
            dev.compact(streams, case["max"], case["flags"])
        assert (ei.value.code, ei.value.message) == (exp["error_code"], exp["message"])
        return
    runs, info = dev.compact(streams, case["max"], case["flags"], with_info=True)
    if "dropped_tables" in exp:
        assert info["dropped_tables"] == exp["dropped_tables"]
    assert [r.table_id for r in runs] == [e.get("table_id", 0) for e in exp["runs"]]
    assert [r.data.hex() for r in runs] == [e["hex"] for e in exp["runs"]]
    assert [(r.stats.size_bytes, r.stats.put_count, r.stats.delete_count) for r in runs] == \
        [(e["size_bytes"], e["put_count"], e["delete_count"]) for e in exp["runs"]]
    assert [r.stats.min_key.encode().hex() for r in runs] == [e["min_key"] for e in exp["runs"]]
    assert [r.stats.max_key.encode().hex() for r in runs] == [e["max_key"] for e in exp["runs"]]
    assert hashlib.sha256(b"".join(r.data for r in runs)).hexdigest() == case["sha256"]


def test_wal_with_corrupt_or_unsorted_stream_matches_oracle(dev):
    """WAL split with an undecodable stream: the first failure in k_way::merge's pop order wins --
    the decode error (raised after its stream's last decodable record is popped), a bad WAL key
    (wal_compaction.rs:71-79) or a failed send to a table whose task died on an order error
    (:157-161, the 101st op after it). Unsorted WAL streams follow the heap's exact pop order."""
    good = fmt.encode_run([fmt.put("1.a", b"x"), fmt.put("2.b", b"y")])
    bad_key = fmt.encode_run([fmt.put("1.0", b"x"), fmt.put("nodot", b"y"), fmt.put("3.z", b"y")])
    unsorted = fmt.encode_run([fmt.put("2.c", b"u"), fmt.put("1.b", b"u"), fmt.put("1.d", b"u"), fmt.put("3.a", b"u")])
    cases = [
        [(2, [good]), (1, [good[:-1]])],              # decode error after 1.a
        [(2, [good[:-1]]), (1, [good])],
        [(2, [good]), (1, [bad_key[:-2]])],           # bad key before the decode error
        [(2, [bad_key]), (1, [good[:-3]])],           # decode error (after 1.a) before the bad key
        [(3, [unsorted]), (1, [good])],               # unsorted, no error: heap order, table drops
        [(3, [unsorted]), (1, [good[:-1]])],          # unsorted + decode error
        [(5, [good]), (4, [unsorted]), (2, [bad_key])],
    ]
    # a table whose build fails on its first op pair, then 99..103 more ops of it (the 101st send fails)
    for extra in (99, 100, 101, 103):
        keys = sorted(["+5.b", "05.a"] + [f"5.{i:04d}" for i in range(extra)] + ["6.q"])
        cases.append([(1, [fmt.encode_run([fmt.put(k, b"v") for k in keys])])])
        cases.append([(2, [fmt.encode_run([fmt.put(k, b"v") for k in keys])]), (1, [good[:-1]])])
    bad = []
    for i, streams in enumerate(cases):
        exp, got = _run_both(dev, streams, 4 * MiB, _abi.SKV_SPLIT_BY_TABLE)
        if exp != got:
            bad.append((i, _diff(exp, got), exp[:3] if exp[0] == "err" else "ok", got[:3] if got[0] == "err" else "ok"))
    assert not bad, bad


def test_drop_tombstones_with_unsorted_stream_matches_oracle(dev):
    """SKV_DROP_TOMBSTONES with a key decrease: build_runs' order check sees only what the filter
    let through (table_tree_compaction.rs:139-147), in the heap's pop order -- a decrease among
    Deletes passes, one among Puts fails, and decode errors compete by pop position."""
    r = random.Random(31)
    cases = []
    for trial in range(150):
        streams = []
        for s in range(r.randint(1, 6)):
            keys = sorted({f"k{r.randrange(60):03d}" for _ in range(r.randint(0, 25))})
            for _ in range(r.randint(0, 2)):  # swap neighbours: decreases
                if len(keys) > 1:
                    i = r.randrange(len(keys) - 1)
                    keys[i], keys[i + 1] = keys[i + 1], keys[i]
            ops = [fmt.delete(k) if r.random() < 0.5 else fmt.put(k, bytes([r.randrange(256)]) * r.randrange(4))
                   for k in keys]
            run = fmt.encode_run(ops)
            if r.random() < 0.15 and len(run) > 2:
                run = run[: r.randrange(1, len(run))]
            members = [run] if r.random() < 0.8 else [run, fmt.encode_run([fmt.put("zz%d" % s, b"m")])]
            streams.append((s * 7 + 1, members))
        cases.append(streams)
    bad, n_ok = [], 0
    for i, streams in enumerate(cases):
        exp, got = _run_both(dev, streams, r.choice([40, 4 * MiB]), _abi.SKV_DROP_TOMBSTONES)
        n_ok += exp[0] == "ok"
        if exp != got:
            bad.append((i, _diff(exp, got)))
    assert not bad, bad[:5]
    assert n_ok > 20  # some unsorted inputs succeed: their decreases were all among Deletes


def test_heap_order_on_the_record_sort_path(dev):
    """Heap-order mode through the record sort (more than 1536 streams): unsorted WAL streams and
    the Delete filter over 1,700 streams."""
    r = random.Random(47)
    for flags in (_abi.SKV_SPLIT_BY_TABLE, _abi.SKV_DROP_TOMBSTONES):
        streams = []
        for s in range(1700):
            keys = sorted({f"{r.randrange(4)}.{r.randrange(400):04d}" for _ in range(r.randint(0, 6))})
            if len(keys) > 1 and r.random() < 0.02:
                keys[0], keys[-1] = keys[-1], keys[0]
            ops = [fmt.delete(k) if r.random() < 0.3 else fmt.put(k, b"v%d" % s) for k in keys]
            streams.append((s + 1, [fmt.encode_run(ops)] if ops else []))
        exp, got = _run_both(dev, streams, 4 * MiB, flags)
        assert exp == got, _diff(exp, got)
        assert dev.timings()["sorted"] == 1


def test_run_count_equal_to_streams_without_one_run_each(dev):
    """Past the splitter fan-in, the device-built run tables take the run record bases as the stream
    bases; that holds only with one run per stream. An empty stream beside a two-member stream also
    has as many runs as streams: such calls must keep the host tables, so a key decrease or a decode
    error after the two-member stream is still reported as the oracle reports it."""
    r = random.Random(61)
    base = []
    for s in range(1700):
        ks = sorted(r.sample(range(10**6), 4))
        base.append([fmt.put(f"{k:06d}{s:04d}", bytes([s & 255]) * 8) for k in ks])
    for case in ("ok", "decrease", "decode"):
        streams = []
        for s, ops in enumerate(base):
            if s == 5:
                streams.append((10**6 - s, []))  # the empty stream
            elif s == 9:  # two members, ascending across the members
                streams.append((10**6 - s, [fmt.encode_run(ops[:2]), fmt.encode_run(ops[2:])]))
            elif s == 40 and case == "decrease":
                streams.append((10**6 - s, [fmt.encode_run([ops[1], ops[0]] + ops[2:])]))
            elif s == 40 and case == "decode":
                streams.append((10**6 - s, [fmt.encode_run(ops)[:-3]]))
            else:
                streams.append((10**6 - s, [fmt.encode_run(ops)]))
        assert sum(len(m) for _, m in streams) == len(streams)
        for flags in (0, _abi.SKV_SPLIT_BY_TABLE):
            exp, got = _run_both(dev, streams, 4 * MiB, flags)
            assert exp == got, (case, flags, _diff(exp, got))


def test_wal_split_matches_oracle(dev):
    """WAL compaction (wal_compaction.rs:66-174) on device: table split, prefix strip (incl. the
    format!("{id}.") length quirk), one run per table, swallowed failing tables, bad keys."""
    r = random.Random(17)
    bad = []
    n = 0
    for trial in range(120):
        n_streams = r.randint(1, 16)
        tables = [r.choice(["7", "-3", "12", "007", "+5", "0", "9223372036854775807", "-9223372036854775808"])
                  for _ in range(r.randint(1, 5))]
        streams = []
        for s in range(n_streams):
            keys = sorted({f"{r.choice(tables)}.{r.randrange(10**4):04d}" for _ in range(r.randint(0, 60))})
            if r.random() < 0.05:
                keys = sorted(set(keys) | {r.choice(["nodot", "x.1", ".5", "99999999999999999999.z", "-.q"])})
            ops = [fmt.put(k, bytes(r.randrange(256) for _ in range(r.randrange(0, 12)))) if r.random() < .85
                   else fmt.delete(k) for k in keys]
            streams.append((s + 1, [fmt.encode_run(ops)] if ops else []))
        max_size = r.choice([40, 200, 1000, 4 * MiB])
        exp, got = _run_both(dev, streams, max_size, _abi.SKV_SPLIT_BY_TABLE)
        n += 1
        if exp != got:
            bad.append((trial, _diff(exp, got)))
    assert not bad, bad[:5]


def test_wal_one_pass_stage(dev):
    """The one-pass WAL stage (k_wal_fused) where it applies -- sorted streams, good keys, ascending
    stripped keys, every table within max -- and the exact stage where it declines: many tables across
    many 512-record workgroups, short and long records (output staged in LDS, or composed from the
    record lines where a workgroup's span is past the stage), Deletes, tables of one record, a table over
    max, a bad key, "007.a"
    next to "7.0" (one table whose stripped keys decrease). Every outcome equal to the oracle's."""
    r = random.Random(29)
    tables = [str(t) for t in range(-40, 300)]
    streams = []
    for s in range(12):
        keys = sorted({f"{r.choice(tables)}.{r.randrange(10**6):06d}" for _ in range(2500)})
        # short and long records mixed (a workgroup's output span past k_wal_fused's block table too)
        ops = [fmt.put(k, bytes(r.randrange(256) for _ in range(r.randrange(0, 20) if r.random() < .8
                                                                 else r.randrange(50, 300))))
               if r.random() < .9 else fmt.delete(k) for k in keys]
        streams.append((s + 1, [fmt.encode_run(ops)]))
    single = [(100, [fmt.encode_run([fmt.put("777.x", b"only")])])]
    # long records only: every workgroup's span is past the LDS stage and the block table (the
    # pieces are composed from the record lines, a binary search per block)
    longs = []
    for s in range(3):
        keys = sorted({f"{r.choice(tables)}.{r.randrange(10**6):06d}" for _ in range(1500)})
        longs.append((50 + s, [fmt.encode_run([fmt.put(k, bytes(r.randrange(256) for _ in range(r.randrange(150, 400))))
                                               for k in keys])]))
    for sts, max_size, stage in ((streams, 4 * MiB, 1), (streams + single, 4 * MiB, 1), (streams, 600, 2),
                                 (longs, 64 * MiB, 1)):
        exp, got = _run_both(dev, sts, max_size, _abi.SKV_SPLIT_BY_TABLE)
        assert exp == got, _diff(exp, got)
        assert dev.timings()["wal_stage"] == stage
    bad_key = [(101, [fmt.encode_run([fmt.put("5.a", b"1"), fmt.put("nodot", b"2")])])]
    quirk = [(102, [fmt.encode_run([fmt.put("007.a", b"1")])]), (103, [fmt.encode_run([fmt.put("7.0", b"2")])])]
    for sts in (streams + bad_key, quirk):  # (quirk alone: the two keys must be neighbours in merged order)
        exp, got = _run_both(dev, sts, 4 * MiB, _abi.SKV_SPLIT_BY_TABLE)
        assert exp == got, _diff(exp, got)
        assert dev.timings()["wal_stage"] == 2
    old = knob_get("SKV_WAL_FUSED")
    knob("SKV_WAL_FUSED", "0")
    try:
        exp, got = _run_both(dev, streams, 4 * MiB, _abi.SKV_SPLIT_BY_TABLE)
        assert exp == got, _diff(exp, got)
        assert dev.timings()["wal_stage"] == 2
    finally:
        if old is None:
            knob("SKV_WAL_FUSED", None)
        else:
            knob("SKV_WAL_FUSED", old)


def test_chain_window_predicted_past_the_end(dev):
    """k_chain (the single-wave greedy split) with records above max among small ones: near the end
    of the merged records a run's predicted window lies wholly past the last record, and its
    fallback search must stay inside P[0..K] -- it used to read past the end and close the last run
    too late (one 36-record, 41,837-byte run at max 900). The input is the key range where the
    general host pipeline's part 2 met it: five streams of 26 / 916 / 3,016-byte records cut to one
    key range, plus the previous range's last output run at the lowest SeqNo."""
    rng = random.Random(17)
    ops_by_stream = []
    for s in range(5):
        ids = sorted(rng.sample(range(3000), 400))
        ops_by_stream.append([fmt.put(f"r{i:06d}", bytes([s]) * rng.choice([10, 900, 3000])) for i in ids])
    keys = sorted({op[1] for ops in ops_by_stream for op in ops})
    cuts = [None] + [keys[p * len(keys) // 6] for p in range(1, 6)] + [None]
    carry = None
    for p in range(6):
        lo, hi = cuts[p], cuts[p + 1]
        sts = [(s + 1, [fmt.encode_run([op for op in ops if (lo is None or op[1] >= lo) and (hi is None or op[1] < hi)])])
               for s, ops in enumerate(ops_by_stream)]
        if carry is not None:
            sts.append((-100, [carry]))
        for mx in (900, 2500):
            exp, got = _run_both(dev, sts, mx, 0)
            assert exp == got, (p, mx, _diff(exp, got))
        carry = pyoracle.compact(sts, 900, 0)[-1].data


def test_greedy_split_random_sizes_with_oversized_records(dev):
    """build_runs' greedy split (runs.rs:211-238) where records above max sit among small ones:
    300 random inputs (record sizes 10 B to 4 KB in runs of similar sizes, max 20 B to 6 KB), each
    equal to the oracle -- the single-wave chain's windows, its fallback searches near the end and
    the one-record runs of oversized records."""
    r = random.Random(53)
    bad = []
    for seed in range(300):
        streams = []
        for s in range(r.randint(1, 6)):
            n = r.randint(0, 600)
            keys = sorted(r.sample(range(5000), n))
            sizes = [r.choice([1, 5, 30, 200, 900, 3000]) for _ in range(3)]
            streams.append((s + 1, [fmt.encode_run([fmt.put(f"q{k:05d}", bytes([s]) * r.choice(sizes)) for k in keys])]))
        mx = r.choice([20, 100, 500, 900, 1500, 3000, 6000])
        exp, got = _run_both(dev, streams, mx, 0)
        if exp != got:
            bad.append((seed, mx, _diff(exp, got)))
    assert not bad, bad[:5]


@pytest.mark.parametrize("max_size", [(1 << 64) - 1, (1 << 64) - 2, (1 << 63) + 5])
@pytest.mark.parametrize("flags", [0, _abi.SKV_DROP_TOMBSTONES], ids=["flags0", "drop"])
def test_max_run_size_near_two_to_the_64(dev, max_size, flags):
    """build_runs compares u64 sizes without overflow (runs.rs:219): with max near 2^64 every record
    joins one run. The chain's byte budget P[b] + max - 1 and its byte-table windows saturate
    instead of wrapping: variable sizes (the general split), one size (arithmetic) and
    the fused shape."""
    streams = gen.config3(seed=4242, n_streams=10, run_bytes=64 * 1024)
    exp, got = _run_both(dev, streams, max_size, flags)
    assert exp == got, _diff(exp, got)
    r = random.Random(17)
    fixed = [(s + 1, [fmt.encode_run([fmt.put(f"k{k:07d}", bytes([s]) * 40)
                                      for k in sorted(r.sample(range(50000), 3000))])]) for s in range(5)]
    exp, got = _run_both(dev, fixed, max_size, flags)
    assert exp == got, _diff(exp, got)


def test_wal_one_pass_stage_many_tables(dev):
    """k_wal_fused's table-start list past the readback it reads with the verdict (WF_GUESS = 1024
    starts: the rest comes in a second copy) and past its capacity (WF_TCAP = 65536: the exact stage
    runs). Tables of one to three records, spread over several streams and many 512-record
    workgroups; the descriptors' min/max key offsets come from the list, so both are compared with
    the oracle byte for byte."""
    r = random.Random(31)
    for n_tables, stage in ((3000, 1), (70000, 2)):
        recs = {}
        for t in range(n_tables):
            for _ in range(1 if n_tables > 65536 else r.randint(1, 3)):
                recs[f"{t}.{r.randrange(10**4):04d}"] = r.randrange(4)
        keys = sorted(recs)
        streams = []
        for s in range(4):
            ks = [k for k in keys if recs[k] % 4 == s]
            streams.append((s + 1, [fmt.encode_run([fmt.put(k, bytes([s]) * (1 + len(k) % 5)) for k in ks])]))
        exp, got = _run_both(dev, streams, 4 * MiB, _abi.SKV_SPLIT_BY_TABLE)
        assert exp == got, _diff(exp, got)
        assert dev.timings()["wal_stage"] == stage, (n_tables, dev.timings()["wal_stage"])


def test_wal_config5_shape(dev):
    """Config-5 record shape (32 B keys "{table}.{suffix}", 8 B values) at a 16-run fan-in like
    the reference job (wal_compaction.rs:18), and at 1000 runs."""
    for n_streams in (16, 1000):
        streams = gen.config5(n_streams=n_streams)
        exp, got = _run_both(dev, streams, 4 * MiB, _abi.SKV_SPLIT_BY_TABLE)
        assert exp == got, _diff(exp, got)


def test_random_cases_match_oracle(dev):
    """The oracle-vs-pyref domain (corrupt runs, unsorted streams, dups, tombstones, tiny max sizes,
    WAL splits) through the GPU path: every seed equal. WAL tables whose failed task races with
    1..100 later sends (the reference may or may not report "Failed to send operation to table
    channel") are resolved the same way by oracle and device, and counted."""
    import pyref

    bad = []
    racy = 0
    for seed in range(600):
        streams, max_size, flags = _case(seed)
        exp, got = _run_both(dev, streams, max_size, flags)
        races = []
        try:
            pyref.compact(streams, max_size, flags, races)
        except pyref.Err:
            pass
        racy += bool(races)
        if exp != got:
            bad.append((seed, _diff(exp, got)))
    print(f"600 seeds, {racy} with a WAL send race window")
    assert not bad, f"{len(bad)} mismatches, first: {bad[:5]}"


@pytest.mark.parametrize("name,streams,max_size,flags", [
    ("cfg1_full", lambda: gen.config1(), 4 * MiB, 0),
    ("cfg2A_scaled", lambda: gen.config2(n_streams=64, n_records=3000, vsize=256), 4 * MiB, 0),
    ("cfg2B_scaled", lambda: gen.config2(n_streams=64, n_records=3000, vsize=256, variant="B"), 4 * MiB, 0),
    ("cfg2A_small_runs", lambda: gen.config2(n_streams=16, n_records=2000, vsize=40), 64 * KiB, 0),
    ("cfg3_scaled", lambda: gen.config3(n_streams=32, run_bytes=192 * KiB), 256 * KiB, 0),
    ("cfg3_scaled_drop", lambda: gen.config3(n_streams=32, run_bytes=192 * KiB), 256 * KiB, 1),
    ("cfg3_256way", lambda: gen.config3(n_streams=256, run_bytes=24 * KiB, vsize=64), 1 * MiB, 0),
    # 256 streams x ~295 records: two sample levels
    ("cfg3_256way_levels", lambda: gen.config3(n_streams=256, run_bytes=96 * KiB, vsize=64), 1 * MiB, 0),
    ("two_streams_big", lambda: gen.config2(n_streams=2, n_records=40000, vsize=100, variant="B"), 4 * MiB, 0),
    ("one_stream", lambda: gen.config2(n_streams=1, n_records=50000, vsize=20), 1 * MiB, 0),
])
def test_generated_configs_match_oracle(dev, name, streams, max_size, flags):
    s = streams()
    exp, got = _run_both(dev, s, max_size, flags)
    assert exp == got, _diff(exp, got)


def test_l0_concatenation_many_members(dev):
    """buffer runs + a 40-member L0 stream at SeqNo 0 (table_buffer_compaction.rs:67-100)."""
    r = random.Random(7)
    l0 = []
    for i in range(40):
        keys = sorted({f"k{i:03d}{r.randrange(10**6):06d}" for _ in range(300)})
        l0.append(fmt.encode_run([fmt.put(k, bytes(r.randrange(256) for _ in range(r.randrange(0, 90)))) for k in keys]))
    bufs = []
    for s in range(1, 9):
        keys = sorted({f"k{r.randrange(40):03d}{r.randrange(10**6):06d}" for _ in range(900)})
        bufs.append((s, [fmt.encode_run([fmt.put(k, b"v%d" % s) if r.random() < .8 else fmt.delete(k) for k in keys])]))
    streams = bufs + [(0, l0)]
    exp, got = _run_both(dev, streams, 256 * KiB, 0)
    assert exp == got, _diff(exp, got)


def test_values_with_fake_records(dev):
    """Values that contain well-formed records defeat the speculative chunk start and force
    the sequential repair (k_fixup)."""
    r = random.Random(3)
    fake = fmt.encode_record(fmt.put("zz", b"x" * 20)) * 40
    streams = []
    for s in range(4):
        keys = sorted({f"key{r.randrange(10**7):07d}" for _ in range(400)})
        ops = [fmt.put(k, fake[: r.randrange(len(fake))]) for k in keys]
        streams.append((s + 1, [fmt.encode_run(ops)]))
    exp, got = _run_both(dev, streams, 1 * MiB, 0)
    assert exp == got, _diff(exp, got)


def test_records_spanning_many_chunks(dev):
    """Values far larger than the 4 KiB walk chunk (pass-through chunks), incl. the reference's
    52 x 1 MiB records at max 2 MiB (runs.rs:914-1000)."""
    ops = []
    for i in range(52):
        key = ("key_%010d" % i).encode()
        ops.append((True, key, bytes(MiB - (1 + 4 + len(key) + 4))))
    runs = dev.compact([(1, [fmt.encode_run(ops)])], 2 * MiB, 0)
    assert len(runs) == 52 and all(r.stats.size_bytes == MiB + 1 for r in runs)
    r = random.Random(5)
    streams = [(s, [fmt.encode_run([fmt.put(f"{s}-{i:04d}", bytes(r.randrange(256) for _ in range(r.randrange(5000, 30000))))
                                    for i in range(40)])]) for s in range(1, 4)]
    exp, got = _run_both(dev, streams, 200 * KiB, 0)
    assert exp == got, _diff(exp, got)


def test_corruption_at_every_position_class(dev):
    """Truncations and flipped bytes across a multi-chunk run: the device reports the same
    first error as the reference decoder."""
    base_ops = [fmt.put(f"k{i:05d}", bytes([i % 251]) * (i % 37)) for i in range(3000)]
    base = fmt.encode_run(base_ops)
    other = fmt.encode_run([fmt.put(f"k{i:05d}x", b"o") for i in range(0, 3000, 7)])
    r = random.Random(11)
    bad = []
    for trial in range(60):
        data = bytearray(base)
        if trial % 2 == 0:
            data = data[: r.randrange(1, len(data))]
        else:
            data[r.randrange(1, len(data))] = r.choice([0, 3, 0xFF, 0xC3, 0x80])
        streams = [(2, [bytes(data)]), (1, [other])]
        exp, got = _run_both(dev, streams, 64 * KiB, 0)
        if exp != got:
            bad.append((trial, _diff(exp, got)))
    assert not bad, bad[:5]


@pytest.mark.parametrize("chunk", [8192, 12288, 16384, 32768, 65536])
def test_longer_speculative_walks(dev, chunk):
    """Big calls walk 8-64 KiB per speculative chunk (skv_compact.hip picks the length from the call
    size); SKV_CHUNK_BYTES forces a length on small inputs: fake records in values, records
    spanning chunks, and corruption everywhere must still give the reference's outcome."""
    old = knob_get("SKV_CHUNK_BYTES")
    knob("SKV_CHUNK_BYTES", str(chunk))
    try:
        test_values_with_fake_records(dev)
        test_records_spanning_many_chunks(dev)
        test_corruption_at_every_position_class(dev)
    finally:
        if old is None:
            knob("SKV_CHUNK_BYTES", None)
        else:
            knob("SKV_CHUNK_BYTES", old)


def test_device_resident_entry_point(dev):
    """skv_compact_dev over HBM-resident inputs returns the same bytes as the host entry point."""
    torch = pytest.importorskip("torch")
    streams = gen.config2(n_streams=8, n_records=5000, vsize=64, variant="B")
    ref = dev.compact(streams, 256 * KiB, 0)
    dev_bufs = [(s, [torch.frombuffer(bytearray(r), dtype=torch.uint8).cuda() for r in runs]) for s, runs in streams]
    torch.cuda.synchronize()
    res = dev.compact_dev([(s, [(t.data_ptr(), t.numel()) for t in ts]) for s, ts in dev_bufs], 256 * KiB, 0)
    out = torch.empty(res.n_bytes, dtype=torch.uint8, device="cuda")
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipMemcpy(ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(res.dev_ptr), ctypes.c_size_t(res.n_bytes), 3) == 0
    blob = bytes(out.cpu().numpy())
    assert blob == b"".join(r.data for r in ref)
    assert [(d[0], d[1]) for d in res.descs] == [(sum(len(x.data) for x in ref[:i]), len(ref[i].data)) for i in range(len(ref))]
    t = dev.timings()
    assert t["gather_ms"] > 0 and t["total_ms"] >= t["gather_ms"]
    res.free()


def test_fixed_stride_fast_path_and_fallback(dev):
    """The single-pass parse taken when every run's first record predicts a fixed stride, and
    its fallback to the general parse when a run breaks the prediction."""
    r = random.Random(21)

    def fixed_run(s, n, corrupt=None):
        keys = sorted({f"{s:02d}{r.randrange(10**12):012d}xy" for _ in range(n)})
        data = bytearray(fmt.encode_run([fmt.put(k, bytes(r.randrange(256) for _ in range(30))) for k in keys]))
        if corrupt is not None:
            data[corrupt] = 0xFF
        return bytes(data)

    cases = []
    # all fixed, clean (fast path end to end)
    cases.append([(s, [fixed_run(s, 500)]) for s in range(1, 9)])
    # all fixed, one run corrupt deep inside (fast path -> fallback -> the reference's error)
    for pos in (1 + 55 * 300 + 0, 1 + 55 * 300 + 7, 1 + 55 * 410 + 21, 1 + 55 * 499 + 30):  # marker, key, val_len, value
        cases.append([(s, [fixed_run(s, 500, corrupt=pos if s == 3 else None)]) for s in range(1, 9)])
    # first record predicts stride 25 and the body is a multiple of it, but sizes vary
    odd = fmt.encode_run([fmt.put("a" * 16, b""), fmt.put("b" * 15, b""), fmt.put("c" * 17, b""), fmt.put("d" * 16, b"")])
    cases.append([(2, [odd]), (1, [fixed_run(1, 100)])])
    # a long variable-size run whose first record size divides its body (the last value padded to
    # make it so): the stride check fails in every chunk, which then walks from a speculative start
    vk = sorted({f"v{r.randrange(10**9):09d}" + "x" * r.randrange(0, 40) for _ in range(3000)})
    vops = [fmt.put(k, bytes(r.randrange(256) for _ in range(r.randrange(0, 120)))) for k in vk]
    first = len(fmt.encode_record(vops[0]))
    body = sum(len(fmt.encode_record(o)) for o in vops)
    pad = (-body) % first
    vops[-1] = fmt.put(vops[-1][1], vops[-1][2] + bytes(pad))
    var_run = fmt.encode_run(vops)
    assert (len(var_run) - 1) % first == 0
    cases.append([(2, [var_run]), (1, [fixed_run(1, 300)])])
    # Puts and Deletes of one size (9 + 16 + 0 == 5 + 20): a valid fixed stride with both markers
    mixed = fmt.encode_run(sorted([fmt.put(f"m{i:015d}", b"") for i in range(0, 400, 2)] +
                                  [fmt.delete(f"m{i:019d}") for i in range(1, 400, 2)], key=lambda o: o[1]))
    cases.append([(2, [mixed]), (1, [fixed_run(1, 100)])])
    # fixed stride, key order violated inside a run (order error from the fast path's check)
    keys = [f"k{i:015d}" for i in range(200)]
    keys[120], keys[121] = keys[121], keys[120]
    cases.append([(1, [fmt.encode_run([fmt.put(k, b"v") for k in keys])]), (2, [fixed_run(2, 50)])])
    # L0-style stream of several fixed members + a variable-size stream (general path)
    cases.append([(0, [fixed_run(7, 80), fixed_run(8, 80)]), (5, [odd])])
    bad = []
    for i, streams in enumerate(cases):
        exp, got = _run_both(dev, streams, 8 * KiB, 0)
        if exp != got:
            bad.append((i, _diff(exp, got)))
    assert not bad, bad


def test_oversized_tile_fallback(dev):
    """Splitter sampling bounds a tile at m*S + k*S records; this input puts 4,606 records in
    one tile (> TILE_CAP 4096), so the global-memory sort path (tile_big) runs, with duplicates
    across streams and Deletes (also under SKV_DROP_TOMBSTONES)."""
    a_keys = [f"k{10 * i + 5:09d}" for i in range(20000)]
    b_keys = ([f"k{0:09d}"] + [f"k{76801 + 20 * i:09d}" for i in range(1535)] +
              [f"k{10 ** 8 + i:09d}" for i in range(1000)])
    b_dup = sorted(set(b_keys) | {f"k{10 * i + 5:09d}" for i in range(7700, 10700, 3)})
    r = random.Random(9)
    for keys_b in (b_keys, b_dup):
        a = fmt.encode_run([fmt.put(k, bytes([r.randrange(256)]) * r.randrange(0, 9)) for k in a_keys])
        b = fmt.encode_run([fmt.delete(k) if r.random() < 0.3 else fmt.put(k, b"new") for k in keys_b])
        for flags in (0, _abi.SKV_DROP_TOMBSTONES):
            exp, got = _run_both(dev, [(1, [a]), (2, [b])], 64 * KiB, flags)
            assert exp == got, _diff(exp, got)


def test_invalid_utf8_key_in_variable_runs(dev):
    """Variable-size runs: the chunk walks check structure only, the emit pass checks each key's
    UTF-8 with the loads that fingerprint it; a bad key reruns the exact walks, whose decode stops
    there (runs.rs:585-591). Valid non-ASCII keys take no rerun."""
    r = random.Random(21)
    for trial in range(6):
        streams = []
        for s in range(5):
            keys = sorted({("k%05d" % r.randrange(10**5)) + "é" * r.randint(0, 3) + "x" * r.randint(0, 40)
                           for _ in range(300)})
            ops = [fmt.put(k, bytes(r.randrange(256) for _ in range(r.randint(0, 30)))) for k in keys]
            run = bytearray(fmt.encode_run(ops))
            if s == trial % 5 and trial < 5:  # corrupt one key byte into an invalid UTF-8 byte
                p = 1
                for _ in range(r.randrange(len(ops))):
                    kl = int.from_bytes(run[p + 1:p + 5], "big")
                    vl = int.from_bytes(run[p + 5 + kl:p + 9 + kl], "big")
                    p += 9 + kl + vl
                run[p + 5 + 1] = 0xFF
            streams.append((s + 1, [bytes(run)]))
        exp, got = _run_both(dev, streams, 1 << 16, 0)
        assert exp == got, _diff(exp, got)


def test_staged_chunk_walks(dev):
    """The chunk walks stage each record's arrays (key prefix, length, Delete bit, fingerprint, ASCII
    bit) for k_emit, which then reads no record (skv_dev.hpp walk_fast<.., true>): records long
    enough that chunks are staged, with non-ASCII keys (k_emit checks their UTF-8), keys past the
    staged limit (144 B: the chunk's staging stops there, k_emit parses it from the records), short
    records among long ones (a chunk past its staged capacity), Deletes, and an invalid UTF-8 key
    (the exact rerun). Every outcome equal to the oracle's."""
    r = random.Random(61)
    for trial in range(8):
        streams = []
        for s in range(6):
            keys = set()
            for _ in range(400):
                kind = r.random()
                tail = ("x" * r.randint(0, 60) if kind < .6 else "é" * r.randint(1, 40) if kind < .85
                        else "y" * r.randint(140, 300))
                keys.add("k%05d" % r.randrange(10**5) + tail)
            ops = []
            for k in sorted(keys):
                if r.random() < .1:
                    ops.append(fmt.delete(k))
                else:
                    # (trial 2: short records only -- chunks past the staged capacity)
                    long_ok = trial != 2 and ((trial & 1) or r.random() < .7)
                    vlen = r.randint(150, 400) if long_ok else r.randint(0, 8)
                    ops.append(fmt.put(k, bytes(r.randrange(256) for _ in range(vlen))))
            run = bytearray(fmt.encode_run(ops))
            if trial >= 6 and s == 2:  # one key byte made invalid UTF-8
                p, i = 1, 0
                target = r.randrange(len(ops))
                while i < target:
                    kl = int.from_bytes(run[p + 1:p + 5], "big")
                    p += 5 + kl + (4 + int.from_bytes(run[p + 5 + kl:p + 9 + kl], "big") if run[p] == 1 else 0)
                    i += 1
                run[p + 5 + 2] = 0xFF
            streams.append((s + 1, [bytes(run)]))
        for flags in (0, _abi.SKV_DROP_TOMBSTONES):
            exp, got = _run_both(dev, streams, 1 << 18, flags)
            assert exp == got, (trial, flags, _diff(exp, got))


def test_coarse_sample_levels_same_bytes(dev):
    """The sample levels above the first only pick splitters: with a 2x or 4x coarser step there
    (SKV_HI_STEP; tiles past TILE_CAP take the oversized-tile path) the output is the same."""
    streams = gen.config3(seed=77, n_streams=300, run_bytes=160 * KiB, vsize=32)
    ref = dev.compact(streams, 1 * MiB, 0)
    for f in ("2", "4"):
        knob("SKV_HI_STEP", f)
        try:
            got = dev.compact(streams, 1 * MiB, 0)
        finally:
            knob("SKV_HI_STEP", None)
        assert [r.data for r in got] == [r.data for r in ref], f


def test_threaded_table_staging(dev):
    """Host tables above SKV_PAR_COPY_MIN bytes are copied into the pinned upload arena by
    several threads (10^6-run calls); forced down to 4 KiB here, a 1000-run WAL call and a
    256-way call still match the oracle."""
    knob("SKV_PAR_COPY_MIN", "4096")
    try:
        for streams, flags in ((gen.config5(n_streams=1000), _abi.SKV_SPLIT_BY_TABLE),
                               (gen.config3(n_streams=256, run_bytes=24 * KiB, vsize=64), 0)):
            exp, got = _run_both(dev, streams, 4 * MiB, flags)
            assert exp == got, _diff(exp, got)
    finally:
        knob("SKV_PAR_COPY_MIN", None)


def test_device_entry_reuse_across_calls(dev):
    """skv_compact_dev lends the ctx's job tables to each call: a 2000-stream call, a call that
    fails in build_job (duplicate seq_no), a failing decode and a small call on one ctx, each
    checked against the oracle."""
    import ctypes

    torch = pytest.importorskip("torch")
    hip = ctypes.CDLL("libamdhip64.so")

    def on_device(streams):
        keep = [(s, [torch.frombuffer(bytearray(r), dtype=torch.uint8).cuda() if len(r) else
                     torch.empty(0, dtype=torch.uint8, device="cuda") for r in runs]) for s, runs in streams]
        torch.cuda.synchronize()
        return keep, [(s, [(t.data_ptr(), t.numel()) for t in ts]) for s, ts in keep]

    def blob(res):
        out = torch.empty(max(1, res.n_bytes), dtype=torch.uint8, device="cuda")
        assert hip.hipMemcpy(ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(res.dev_ptr),
                             ctypes.c_size_t(res.n_bytes), 3) == 0
        return bytes(out[: res.n_bytes].cpu().numpy())

    big = gen.config5(n_streams=2000)
    small = gen.config2(n_streams=3, n_records=500, vsize=16, variant="B")
    dup = [(1, [small[0][1][0]]), (1, [small[1][1][0]])]
    corrupt = [(2, [small[0][1][0][:-3]]), (1, [small[1][1][0]])]
    for streams, flags in ((big, _abi.SKV_SPLIT_BY_TABLE), (dup, 0), (corrupt, 0), (small, 0), (big, 0)):
        keep, dstreams = on_device(streams)
        try:
            exp = pyoracle.compact_bytes(streams, 64 * KiB, flags)
        except _abi.RunError as e:
            exp = ("err", e.code, e.message)
        try:
            res = dev.compact_dev(dstreams, 64 * KiB, flags)
            got = (blob(res), res.descs)
            res.free()
        except _abi.RunError as e:
            got = ("err", e.code, e.message)
        if exp[0] == "err" and exp[1] == _abi.SKV_E_INVALID_ARG:  # API misuse: code only
            assert got[0] == "err" and got[1] == _abi.SKV_E_INVALID_ARG
        else:
            assert got == exp
