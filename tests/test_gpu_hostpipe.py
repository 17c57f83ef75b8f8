"""The pipelined host paths (skv_compact with host inputs, skv_hostpipe.hip): key-range parts whose
H2D, kernels and D2H overlap on three streams -- the fused pipeline (compact_host_pipelined: one
record size, keys <= 16 B) and the general one (compact_host_pipelined_general: variable-length
records and Deletes, the open output run carried into the next part). Outputs must be the
oracle's, byte for byte, whatever the cut keys (parts 2..17, equal keys across streams at the
cuts, empty parts), and a call the device poisons or rejects (a key decrease inside a part or
across a cut, a corrupt run) must end with the oracle's outcome through the serial path.

SKV_HOST_PIPE_MIN=0 lets small inputs take the pipeline; SKV_HOST_PARTS fixes the part count.
`timings()["host_parts"]` says whether the call was pipelined (0: serial).
"""
import os
import random

import numpy as np
import pytest

from skv import _abi
from skv import format as fmt
from skv.api import Compactor

import pyoracle
from test_gpu_parity import _diff, _norm, _run_both
from knobs import knob, knob_get  # noqa: E402

pytestmark = pytest.mark.gpu
MiB = 1 << 20


@pytest.fixture(scope="module")
def dev():
    torch = pytest.importorskip("torch")
    torch.cuda.init()
    c = Compactor(0)
    yield c
    c.close()


@pytest.fixture
def pipe_env():
    old = {k: os.environ.get(k) for k in ("SKV_HOST_PIPE_MIN", "SKV_HOST_PARTS")}
    os.environ["SKV_HOST_PIPE_MIN"] = "0"
    yield
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def _fixed_run(keys, vlen, tag):
    return fmt.encode_run([fmt.put(k, bytes([(tag + i) & 0xFF]) * vlen) for i, k in enumerate(keys)])


def _streams(rng, k, n, space, klen=12, vlen=40, same=False):
    base = sorted(rng.sample(range(space), n)) if same else None
    out = []
    for s in range(k):
        ids = base if same else sorted(rng.sample(range(space), n))
        keys = [f"k{i:0{klen - 1}d}" for i in ids]
        out.append((s + 1, [_fixed_run(keys, vlen, s)]))
    return out


def _check(dev, streams, max_size, flags, parts, expect_pipe=True):
    os.environ["SKV_HOST_PARTS"] = str(parts)
    exp, got = _run_both(dev, streams, max_size, flags)
    assert exp == got, _diff(exp, got)
    hp = dev.timings()["host_parts"]
    if expect_pipe:
        assert hp == parts, f"not pipelined (host_parts={hp})"
    return hp


@pytest.mark.parametrize("parts", [2, 3, 7, 17])
@pytest.mark.parametrize("max_size", [4 * MiB, 1000, 1 << 62])
def test_pipelined_matches_oracle(dev, pipe_env, parts, max_size):
    rng = random.Random(parts * 1000 + max_size % 997)
    streams = _streams(rng, 8, 3000, 12000)
    _check(dev, streams, max_size, 0, parts)


@pytest.mark.parametrize("parts", [2, 5, 16])
def test_pipelined_drop_tombstones(dev, pipe_env, parts):
    rng = random.Random(7 + parts)
    _check(dev, _streams(rng, 6, 2500, 6000), 4 * MiB, _abi.SKV_DROP_TOMBSTONES, parts)


@pytest.mark.parametrize("parts", [2, 9])
def test_identical_streams_equal_keys_at_every_cut(dev, pipe_env, parts):
    rng = random.Random(parts)
    _check(dev, _streams(rng, 16, 2000, 5000, same=True), 64 * 1024, 0, parts)


def test_more_parts_than_distinct_keys(dev, pipe_env):
    """30 distinct keys, repeated inside each stream (non-decreasing runs): the cut keys repeat,
    which leaves parts empty, and equal keys of one stream keep their first record"""
    rng = random.Random(3)
    streams = []
    for s in range(4):
        keys = sorted(f"k{rng.randrange(30):011d}" for _ in range(700))
        streams.append((s + 1, [_fixed_run(keys, 40, s)]))
    _check(dev, streams, 4 * MiB, 0, 40)


def test_single_stream_and_seq_orders(dev, pipe_env):
    rng = random.Random(11)
    one = _streams(rng, 1, 5000, 9000)
    _check(dev, one, 8192, 0, 6)
    many = _streams(rng, 12, 1500, 4000)
    _check(dev, list(reversed(many)), 8192, 0, 4)  # seq_nos descending in the caller's vector
    shuffled = many[:]
    rng.shuffle(shuffled)
    _check(dev, shuffled, 8192, 0, 4)


@pytest.mark.parametrize("seed", range(6))
def test_decrease_falls_back_to_the_serial_path_with_the_oracles_error(dev, pipe_env, seed):
    rng = random.Random(100 + seed)
    streams = _streams(rng, 5, 2000, 8000)
    s = rng.randrange(5)
    run = bytearray(streams[s][1][0])
    S = (len(run) - 1) // 2000
    i = rng.randrange(1, 2000)  # swap records i-1 and i: one decrease
    a, b = 1 + (i - 1) * S, 1 + i * S
    run[a:a + S], run[b:b + S] = run[b:b + S], run[a:a + S]
    streams[s] = (streams[s][0], [bytes(run)])
    os.environ["SKV_HOST_PARTS"] = str(rng.choice([2, 4, 8]))
    exp, got = _run_both(dev, streams, 4 * MiB, 0)
    assert exp == got and exp[0] == "err", _diff(exp, got)
    assert dev.timings()["host_parts"] == 0


def test_not_eligible_inputs_stay_serial(dev, pipe_env):
    """a WAL flush whose tables break the one-run rule (each over max: dropped) and an L0-style stream
    whose member runs overlap (not one sorted stream) end on the serial path with the oracle's outcome"""
    rng = random.Random(5)
    streams = []
    for s in range(4):
        keys = sorted(rng.sample(range(9000), 1500))
        streams.append((s + 1, [fmt.encode_run([fmt.put(f"{s % 3}.k{i:06d}", b"v" * (1 + i % 7)) for i in keys])]))
    _check(dev, streams, 1000, _abi.SKV_SPLIT_BY_TABLE, 4, expect_pipe=False)
    assert dev.timings()["host_parts"] == 0
    # member runs in descending key order ("1.*" before "0.*"): the concatenation decreases
    l0 = [(1, [streams[1][1][0], streams[0][1][0]])] + streams[2:]
    _check(dev, l0, 1000, 0, 4, expect_pipe=False)
    assert dev.timings()["host_parts"] == 0
    # in ascending order it is one sorted stream, and pipelines
    l0 = [(1, [streams[0][1][0], streams[1][1][0]])] + streams[2:]
    _check(dev, l0, 1000, 0, 4)


# ---- the general key-range pipeline (variable-length records, Deletes) ------------------------

def _var_streams(rng, k, n, space, del_frac=0.1, same=False, vmax=60):
    base = sorted(rng.sample(range(space), n)) if same else None
    out = []
    for s in range(k):
        ids = base if same else sorted(rng.sample(range(space), n))
        ops = []
        for i in ids:
            key = f"k{i:07d}" + "abcdefghij" * (i % 7)  # 8..78-byte keys
            if rng.random() < del_frac:
                ops.append(fmt.delete(key))
            else:
                ops.append(fmt.put(key, bytes([(s * 7 + i) & 0xFF]) * rng.randint(0, vmax)))
        out.append((s + 1, [fmt.encode_run(ops)]))
    return out


@pytest.mark.parametrize("parts", [2, 3, 7, 17])
@pytest.mark.parametrize("max_size", [1000, 4096, 20000])
def test_general_pipeline_matches_oracle(dev, pipe_env, parts, max_size):
    rng = random.Random(parts * 31 + max_size)
    streams = _var_streams(rng, 9, 2500, 15000)
    _check(dev, streams, max_size, 0, parts)


@pytest.mark.parametrize("parts", [2, 5, 16])
def test_general_pipeline_drop_tombstones(dev, pipe_env, parts):
    rng = random.Random(70 + parts)
    streams = _var_streams(rng, 7, 3000, 9000, del_frac=0.3)
    _check(dev, streams, 4096, _abi.SKV_DROP_TOMBSTONES, parts)


@pytest.mark.parametrize("parts", [2, 9])
def test_general_pipeline_equal_keys_at_every_cut(dev, pipe_env, parts):
    rng = random.Random(90 + parts)
    _check(dev, _var_streams(rng, 12, 1500, 4000, same=True), 2048, 0, parts)


def test_general_pipeline_one_record_runs_and_large_records(dev, pipe_env):
    """records larger than max (each its own run) and max sizes just above one record"""
    rng = random.Random(17)
    streams = []
    for s in range(5):
        ids = sorted(rng.sample(range(3000), 400))
        streams.append((s + 1, [fmt.encode_run([fmt.put(f"r{i:06d}", bytes([s]) * rng.choice([10, 900, 3000]))
                                                for i in ids])]))
    for mx in (1, 900, 2500, 8000):
        _check(dev, streams, mx, 0, 6)


@pytest.mark.parametrize("seed", range(6))
def test_general_decrease_inside_or_across_parts_gives_the_oracles_error(dev, pipe_env, seed):
    """a key decrease anywhere (inside a part, or across a cut) ends on the serial path with the
    oracle's outcome"""
    rng = random.Random(300 + seed)
    streams = _var_streams(rng, 5, 2000, 8000, del_frac=0.0)
    s = rng.randrange(5)
    ids = sorted(rng.sample(range(8000), 2000))
    i = rng.randrange(1, 2000)
    ids[i - 1], ids[i] = ids[i], ids[i - 1]
    streams[s] = (streams[s][0], [fmt.encode_run([fmt.put(f"k{x:07d}", b"d") for x in ids])])
    os.environ["SKV_HOST_PARTS"] = str(rng.choice([2, 4, 8]))
    exp, got = _run_both(dev, streams, 4096, 0)
    assert exp == got and exp[0] == "err", _diff(exp, got)


def test_general_corrupt_run_gives_the_oracles_error(dev, pipe_env):
    rng = random.Random(41)
    streams = _var_streams(rng, 4, 1500, 6000)
    bad = bytearray(streams[2][1][0])
    bad[len(bad) // 2] = 0x07  # likely inside a value or a length: some decode error or a changed record
    streams[2] = (streams[2][0], [bytes(bad)])
    truncated = streams[1][1][0][:-3]
    streams[1] = (streams[1][0], [truncated])
    os.environ["SKV_HOST_PARTS"] = "5"
    exp, got = _run_both(dev, streams, 4096, 0)
    assert exp == got, _diff(exp, got)
    assert dev.timings()["host_parts"] == 0


def test_general_pipeline_failure_leaves_the_ctx_clean(dev, pipe_env):
    rng = random.Random(43)
    streams = _var_streams(rng, 6, 2000, 9000)
    os.environ["SKV_HOST_PARTS"] = "5"
    _check(dev, streams, 4096, 0, 5)
    for _ in range(2):
        _check(dev, streams, 4096, 0, 5)


def test_config2_shape_large(dev, pipe_env):
    """64 streams of 281-byte records (BASELINE config 2's record), 20k records each (~360 MB)"""
    rng = np.random.default_rng(2)
    streams = []
    for s in range(64):
        ids = np.sort(rng.choice(2_000_000, 20_000, replace=False))
        rec = np.empty((20_000, 281), np.uint8)
        rec[:, 0] = 1
        rec[:, 1:5] = np.frombuffer((16).to_bytes(4, "big"), np.uint8)
        keys = np.char.encode(np.char.mod("key%013d", ids), "ascii").view(np.uint8).reshape(-1, 16)
        rec[:, 5:21] = keys
        rec[:, 21:25] = np.frombuffer((256).to_bytes(4, "big"), np.uint8)
        rec[:, 25:] = rng.integers(0, 256, (20_000, 256), dtype=np.uint8)
        streams.append((s + 1, [b"\x01" + rec.tobytes()]))
    _check(dev, streams, 4 * MiB, 0, 16)


@pytest.mark.parametrize("fail_at", [0, 1, 3])
def test_failure_mid_pipeline_leaves_the_ctx_clean(dev, pipe_env, fail_at):
    """A failure after some parts were queued (SKV_TEST_FAIL_PART) ends the call with
    SKV_E_DEVICE and its text; the copies it had issued are drained and its pinned output goes
    back to the pool, so the next calls on the same ctx (pipelined and serial) are exact."""
    rng = random.Random(40 + fail_at)
    streams = _streams(rng, 8, 3000, 12000)
    os.environ["SKV_HOST_PARTS"] = "6"
    knob("SKV_TEST_FAIL_PART", str(fail_at))
    try:
        with pytest.raises(_abi.RunError) as ei:
            dev.compact(streams, 4 * MiB, 0)
    finally:
        knob("SKV_TEST_FAIL_PART", None)
    assert ei.value.code == _abi.SKV_E_DEVICE and "injected failure" in ei.value.message
    for _ in range(3):  # the pool's buffer is taken and given back again on every call
        _check(dev, streams, 4 * MiB, 0, 6)
    _check(dev, _streams(rng, 3, 500, 4000), 4 * MiB, 0, 4)


@pytest.mark.parametrize("parts", [3, 8])
def test_general_pipeline_pinned_inputs_kernel_ingest(dev, pipe_env, parts):
    """runs in pinned, device-mapped host memory: with SKV_INGEST=kernel the GPU copies each part's
    slices itself (k_ingest, one launch per part), by default one DMA copy per slice -- also with
    run buffers at odd host offsets"""
    torch = pytest.importorskip("torch")
    rng = random.Random(500 + parts)
    streams = _var_streams(rng, 10, 2500, 12000, del_frac=0.15)
    pinned, pstreams = [], []
    for i, (seq, runs) in enumerate(streams):
        r = runs[0]
        skew = (i * 5) % 16  # host buffers not 16-byte aligned
        t = torch.empty(len(r) + skew, dtype=torch.uint8).pin_memory()
        t[skew:] = torch.frombuffer(bytearray(r), dtype=torch.uint8)
        pinned.append(t)
        pstreams.append((seq, [(t.data_ptr() + skew, len(r))]))
    os.environ["SKV_HOST_PARTS"] = str(parts)
    for mode, mx in (("kernel", 2048), ("kernel", 20000), ("dma", 2048)):
        knob("SKV_INGEST", mode)
        try:
            got = dev.compact_host_ptrs(pstreams, mx, 0, with_runs=True)
        finally:
            knob("SKV_INGEST", None)
        assert dev.timings()["host_parts"] == parts
        exp = pyoracle.compact(streams, mx, 0)
        assert [r.data for r in got] == [r.data for r in exp]
        assert [(r.stats.min_key, r.stats.max_key, r.stats.put_count, r.stats.delete_count) for r in got] == \
            [(r.stats.min_key, r.stats.max_key, r.stats.put_count, r.stats.delete_count) for r in exp]


# ---- real job shapes: L0 / next-level concatenations, WAL flushes ---------------------------------

def _check_pipe(dev, streams, max_size, flags, parts, min_parts=2):
    """as _check, but the part count may come out lower than asked (WAL cuts are distinct tables)"""
    os.environ["SKV_HOST_PARTS"] = str(parts)
    exp, got = _run_both(dev, streams, max_size, flags)
    assert exp == got, _diff(exp, got)
    hp = dev.timings()["host_parts"]
    assert min_parts <= hp <= parts, f"host_parts={hp}"
    return hp


def _l0_stream(rng, n_members, per, space, fixed, seq=0, vmax=60):
    """one stream of n_members ascending, non-overlapping member runs (the L0 concatenation of
    table_buffer_compaction.rs:66-100 at SeqNo 0)"""
    ids = sorted(rng.sample(range(space), n_members * per))
    members = []
    for i in range(n_members):
        chunk = ids[i * per:(i + 1) * per]
        if fixed:
            members.append(_fixed_run([f"k{x:011d}" for x in chunk], 40, 200 + i))
        else:
            ops = [fmt.put(f"k{x:07d}" + "abcdefghij" * (x % 7), bytes([i & 0xFF]) * rng.randint(0, vmax))
                   if rng.random() < .9 else fmt.delete(f"k{x:07d}" + "abcdefghij" * (x % 7)) for x in chunk]
            members.append(fmt.encode_run(ops))
    return (seq, members)


@pytest.mark.parametrize("parts", [2, 5, 11])
def test_fused_pipeline_l0_concatenation_across_cuts(dev, pipe_env, parts):
    """buffer streams + one stream of 40 ascending L0 member runs (one record size: the fused
    pipeline); the cuts fall inside and between member runs"""
    rng = random.Random(600 + parts)
    streams = [(s + 1, [_fixed_run([f"k{x:011d}" for x in sorted(rng.sample(range(40000), 1500))], 40, s)])
               for s in range(6)]
    streams.append(_l0_stream(rng, 40, 150, 40000, fixed=True))
    _check(dev, streams, 4 * MiB, 0, parts)
    _check(dev, streams, 3000, 0, parts)


@pytest.mark.parametrize("parts", [2, 6, 13])
def test_general_pipeline_l0_concatenation_across_cuts(dev, pipe_env, parts):
    """variable-length records and Deletes: buffer streams + an L0 concatenation (25 member runs,
    one of them empty) + a next-level concatenation at another SeqNo (table_tree_compaction.rs:
    103-135); flags 0 and the Delete filter"""
    rng = random.Random(700 + parts)
    streams = _var_streams(rng, 5, 1500, 30000)
    l0 = _l0_stream(rng, 25, 120, 30000, fixed=False, seq=0)
    l0[1].insert(7, b"\x01")  # a member of only a version byte yields nothing
    streams.append(l0)
    streams.append(_l0_stream(rng, 9, 300, 30000, fixed=False, seq=-5))
    for flags in (0, _abi.SKV_DROP_TOMBSTONES):
        _check(dev, streams, 4096, flags, parts)


def _wal_streams(rng, k, n, tables, vmax=30, dels=0.1):
    out = []
    for s in range(k):
        keys = sorted({f"{rng.choice(tables)}.{rng.randrange(10 ** 7):07d}" for _ in range(n)})
        out.append((s + 1, [fmt.encode_run([fmt.put(x, bytes([s]) * rng.randint(0, vmax)) if rng.random() >= dels
                                            else fmt.delete(x) for x in keys])]))
    return out


@pytest.mark.parametrize("parts", [2, 4, 9])
def test_wal_flush_pipelined_across_table_cuts(dev, pipe_env, parts):
    """a WAL flush (wal_compaction.rs:18-174) of 16 WAL runs over 300 tables (negative ids too):
    parts cut at canonical table prefixes, each part's tables whole, the one-pass WAL stage per part;
    output bytes, descriptors (table ids) and dropped-table count equal to the oracle's"""
    rng = random.Random(800 + parts)
    streams = _wal_streams(rng, 16, 2500, [str(t) for t in range(-20, 280)])
    _check_pipe(dev, streams, 4 * MiB, _abi.SKV_SPLIT_BY_TABLE, parts)
    assert dev.timings()["wal_stage"] == 1


def test_wal_flush_pipeline_declines_to_the_serial_path(dev, pipe_env):
    """what a part cannot decide alone ends the attempt, and the serial path gives the oracle's
    outcome: a non-canonical prefix ("007." is table 7, far from "7." in key order), a table over
    max (dropped by the one-run rule), a key without a table prefix (the job fails)"""
    rng = random.Random(901)
    base = _wal_streams(rng, 8, 2000, [str(t) for t in range(100)])
    cases = [
        base + [(50, [fmt.encode_run([fmt.put("007.a", b"x")])])],
        base,  # at max 600 some tables exceed max
        base + [(51, [fmt.encode_run([fmt.put("nodot", b"y")])])],
    ]
    for streams, mx in zip(cases, (4 * MiB, 600, 4 * MiB)):
        os.environ["SKV_HOST_PARTS"] = "4"
        exp, got = _run_both(dev, streams, mx, _abi.SKV_SPLIT_BY_TABLE)
        assert exp == got, _diff(exp, got)
        assert dev.timings()["host_parts"] == 0


def test_wal_flush_of_many_tiny_runs_kernel_ingest(dev, pipe_env):
    """config 5's shape at small scale: 20,000 WAL runs of 10 records in pinned, device-mapped host
    memory -- more slices than one DMA copy each is worth, so the GPU copies each part's slices
    itself (k_ingest_slices); outputs equal to the oracle's"""
    torch = pytest.importorskip("torch")
    rng = random.Random(902)
    tables = [str(t) for t in range(64)]
    runs = []
    for s in range(20000):
        keys = sorted({f"{rng.choice(tables)}.{rng.randrange(10 ** 9):09d}" for _ in range(10)})
        runs.append(fmt.encode_run([fmt.put(x, bytes([s & 0xFF]) * 8) for x in keys]))
    blob = b"".join(runs)
    t = torch.empty(len(blob), dtype=torch.uint8).pin_memory()
    t[:] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    offs = np.cumsum([0] + [len(r) for r in runs[:-1]])
    pstreams = [(s + 1, [(t.data_ptr() + int(o), len(r))]) for s, (o, r) in enumerate(zip(offs, runs))]
    os.environ["SKV_HOST_PARTS"] = "4"
    got = dev.compact_host_ptrs(pstreams, 1 << 40, _abi.SKV_SPLIT_BY_TABLE, with_runs=True)
    assert 2 <= dev.timings()["host_parts"] <= 4
    exp = pyoracle.compact([(s + 1, [r]) for s, r in enumerate(runs)], 1 << 40, _abi.SKV_SPLIT_BY_TABLE)
    assert [r.data for r in got] == [r.data for r in exp]
    assert [r.table_id for r in got] == [r.table_id for r in exp]


def _pinned_wal(torch, runs):
    blob = b"".join(runs)
    t = torch.empty(len(blob), dtype=torch.uint8).pin_memory()
    t[:] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    offs = np.cumsum([0] + [len(r) for r in runs[:-1]])
    return t, [(s + 1, [(t.data_ptr() + int(o), len(r))]) for s, (o, r) in enumerate(zip(offs, runs))]


def test_wal_flush_past_the_walk_threshold(dev, pipe_env):
    """more than 2^16 WAL runs take the serial path (the many-run pipeline of round 5 measured slower
    and was removed) even with parts asked for: runs of one record size per run (sizes
    differ between runs), empty runs (a version byte only), Deletes among Puts of the same size, and
    runs that mix record sizes -- every outcome equal to the oracle's."""
    torch = pytest.importorskip("torch")
    rng = random.Random(903)
    tables = [str(t) for t in range(-5, 60)]
    runs = []
    for s in range(70000):
        if s % 9973 == 5:
            runs.append(b"\x01")
            continue
        keys = sorted({f"{rng.choice(tables)}.{rng.randrange(10 ** 6):06d}" for _ in range(rng.randint(1, 6))})
        vl = 3 + s % 5
        runs.append(fmt.encode_run([fmt.put(x + "x" * (11 - len(x)), bytes([s & 0xFF]) * vl) for x in keys]))
    mixed = [fmt.put("3.aaaaaaaaaa", b"vvvv"), fmt.delete("3.aaaaaaaaab"), fmt.put("3.aaaaaaaaac", b"vvvv")]
    runs = runs[:40000] + [fmt.encode_run(mixed)] + runs[40000:]
    os.environ["SKV_HOST_PARTS"] = "5"
    t, pstreams = _pinned_wal(torch, runs)
    got = dev.compact_host_ptrs(pstreams, 1 << 40, _abi.SKV_SPLIT_BY_TABLE, with_runs=True)
    assert dev.timings()["host_parts"] == 0
    exp = pyoracle.compact([(s + 1, [r]) for s, r in enumerate(runs)], 1 << 40, _abi.SKV_SPLIT_BY_TABLE)
    assert _norm(got) == _norm(exp)


@pytest.mark.parametrize("order", ["ascending", "descending", "mixed"])
def test_serial_path_stages_host_contiguous_runs_as_spans(dev, order):
    """the serial host path (SKV_HOST_PIPE=0) stages runs that tile one host buffer with one copy
    per span: the runs of a WAL flush in one numpy buffer, laid out in rank order (ascending
    addresses), against it (descending, as a caller's seq 1..N buffer ranks), or shuffled (spans of
    one run); an empty stream and a run of only a version byte inside the buffer -- bytes,
    descriptors and the dropped-table count equal to the oracle's"""
    rng = random.Random({"ascending": 11, "descending": 12, "mixed": 13}[order])
    streams = _wal_streams(rng, 40, 300, [str(t) for t in range(30)])
    streams[5] = (streams[5][0], [b"\x01"])
    runs = [r[0] for _, r in streams]
    idx = list(range(len(runs)))
    if order == "ascending":
        idx.reverse()  # rank order is seq descending: lay the highest seq first
    elif order == "mixed":
        rng.shuffle(idx)
    buf = np.frombuffer(b"".join(runs[i] for i in idx), dtype=np.uint8).copy()
    offs, at = [0] * len(runs), 0
    for i in idx:
        offs[i] = at
        at += len(runs[i])
    base = buf.ctypes.data
    pstreams = [(seq, [(base + offs[i], len(runs[i]))]) for i, (seq, _) in enumerate(streams)]
    pstreams.append((100, []))
    old = os.environ.get("SKV_HOST_PIPE")
    os.environ["SKV_HOST_PIPE"] = "0"
    try:
        got = dev.compact_host_ptrs(pstreams, 4 * MiB, _abi.SKV_SPLIT_BY_TABLE, with_runs=True)
    finally:
        if old is None:
            os.environ.pop("SKV_HOST_PIPE", None)
        else:
            os.environ["SKV_HOST_PIPE"] = old
    exp = pyoracle.compact(streams + [(100, [])], 4 * MiB, _abi.SKV_SPLIT_BY_TABLE)
    assert _norm(got) == _norm(exp)
