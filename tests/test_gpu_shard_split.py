"""One compaction split across several GPUs by key range (skv_compact_split, skv_split.hip and
skv_hostpipe.hip). On the one-GPU test box the G ctxs are G ctxs of device 0, one host
thread each: the same code as G GPUs (key-range parts dealt round-robin over the ctxs; each part
staged, merged and deduplicated on its ctx and stream; each part's bytes copied D2H to their global
place once every earlier part's output size is known). Two splits:
  - one record size, keys <= 16 B (the fused path): build_runs' split is arithmetic in the global
    survivor index, so only the parts' survivor counts cross between ctxs;
  - anything else (variable-length records, Deletes, the Delete filter): each part's split continues
    the open run the previous part left (Job::carry), a continuation's descriptor merged into the
    run before it.
Outputs must be the oracle's, byte for byte, for any G, any parts per ctx, any max_run_size (runs
of one record, runs over max, run boundaries inside parts and at part edges), equal keys across
streams, streams absent from parts, parts of only tombstones, member-run (L0) streams. Calls a part
finds a data error in (a key decrease, a truncated run) must end with the oracle's outcome through
skv_compact on ctxs[0]. `timings()` on ctxs[0] says which split ran (`host_parts`, `path`).
"""
import os
import random

import pytest

from skv import _abi
from skv import format as fmt
from skv import gen
from skv.api import Compactor, compact_split

import pyoracle
from test_gpu_parity import _diff, _norm

pytestmark = pytest.mark.gpu
MiB = 1 << 20


@pytest.fixture(scope="module")
def ctxs():
    torch = pytest.importorskip("torch")
    torch.cuda.init()
    cs = [Compactor(0) for _ in range(8)]
    yield cs
    for c in cs:
        c.close()


def _fixed_run(keys, vlen, tag):
    return fmt.encode_run([fmt.put(k, bytes([(tag + i) & 0xFF]) * vlen) for i, k in enumerate(keys)])


def _streams(rng, k, n, space, klen=12, vlen=40, same=False):
    base = sorted(rng.sample(range(space), n)) if same else None
    out = []
    for s in range(k):
        ids = base if same else sorted(rng.sample(range(space), n))
        out.append((s + 1, [_fixed_run([f"k{i:0{klen - 1}d}" for i in ids], vlen, s)]))
    return out


def _both(cs, streams, max_size, flags=0):
    try:
        runs, info = pyoracle.compact(streams, max_size, flags, with_result=True)
        exp = ("ok", _norm(runs), info["dropped_tables"])
    except _abi.RunError as e:
        exp = ("err", e.code, e.message)
    try:
        runs, info = compact_split(cs, streams, max_size, flags, with_info=True)
        got = ("ok", _norm(runs), info["dropped_tables"])
    except _abi.RunError as e:
        got = ("err", e.code, e.message)
    return exp, got


def _check(cs, streams, max_size, flags=0, split=True, parts=1, general=False):
    """split: the fused split (exactly G x parts parts); general: the split with the carried open
    run (parts from sampled cut keys: at least 2); neither: skv_compact on ctxs[0]"""
    os.environ["SKV_SPLIT_PARTS"] = str(parts)
    try:
        exp, got = _both(cs, streams, max_size, flags)
    finally:
        os.environ.pop("SKV_SPLIT_PARTS", None)
    assert exp == got, _diff(exp, got)
    t = cs[0].timings()
    hp = t["host_parts"]
    if general:
        assert hp >= 2 and t["path"] == _abi.PATH_GENERAL, f"not the general split ({t})"
    elif split:
        assert hp == len(cs) * parts and t["path"] == _abi.PATH_FUSED, f"not split ({t})"
    else:
        assert hp != len(cs) * parts


@pytest.mark.parametrize("G", [2, 3, 5, 8])
@pytest.mark.parametrize("max_size", [4 * MiB, 1000, 7777, 1 << 62, (1 << 64) - 1])
def test_split_matches_oracle(ctxs, G, max_size):
    rng = random.Random(G * 1009 + max_size % 991)
    _check(ctxs[:G], _streams(rng, 8, 3000, 12000), max_size)


@pytest.mark.parametrize("G,parts", [(2, 3), (4, 4), (3, 7)])
def test_parts_inside_shards(ctxs, G, parts):
    """several key-range parts per shard: survivor numbering chained through the shard's own parts"""
    rng = random.Random(G * 31 + parts)
    _check(ctxs[:G], _streams(rng, 8, 4000, 15000), 3000, parts=parts)


@pytest.mark.parametrize("G", [2, 4, 8])
def test_equal_keys_in_every_stream(ctxs, G):
    """every stream holds the same keys: each key has its newest version in stream 1, and the cuts
    fall between keys, never between versions of one key"""
    rng = random.Random(77 + G)
    _check(ctxs[:G], _streams(rng, 6, 4000, 9000, same=True), 2000)


def test_streams_absent_from_shards(ctxs):
    """streams over disjoint key ranges: most shards see only some streams, some see one"""
    streams = []
    for s in range(6):
        keys = [f"k{s:02d}{i:09d}" for i in range(0, 6000, 3)]
        streams.append((s + 1, [_fixed_run(keys, 24, s)]))
    _check(ctxs[:4], streams, 3333)


def test_member_run_streams(ctxs):
    """an L0 shape: one stream concatenating many disjoint ascending member runs beside buffer
    streams; member runs straddle the shard cuts"""
    rng = random.Random(5)
    ids = sorted(rng.sample(range(200000), 40000))
    members = [_fixed_run([f"k{i:011d}" for i in ids[j:j + 1000]], 32, j) for j in range(0, len(ids), 1000)]
    streams = [(0, members)]
    for s in range(4):
        streams.append((s + 1, [_fixed_run([f"k{i:011d}" for i in sorted(rng.sample(range(200000), 5000))], 32, s)]))
    _check(ctxs[:4], streams, 5000)


def test_drop_tombstones_flag(ctxs):
    rng = random.Random(11)
    _check(ctxs[:3], _streams(rng, 5, 3000, 8000), 4096, flags=_abi.SKV_DROP_TOMBSTONES)


def test_config2_shape_against_one_gpu(ctxs):
    """a config-2B-shape call (16 streams x 20,000 records, 16-B hex keys, 256-B values, ~37 %
    superseded at full size): the oracle's bytes through 8 shards of several parts each"""
    streams = gen.config2(seed=4242, n_streams=16, n_records=20000, vsize=256, variant="B")
    _check(ctxs[:8], streams, 4 * MiB, parts=3)


def test_mixed_record_sizes_take_the_general_split(ctxs):
    """records of several sizes: outside the fused shape, the split with the carried open run"""
    rng = random.Random(3)
    streams = _streams(rng, 4, 2000, 6000)
    ops = [fmt.put(f"k{i:011d}", b"v" * (1 + i % 7)) for i in sorted(rng.sample(range(6000), 1500))]
    streams.append((9, [fmt.encode_run(ops)]))
    _check(ctxs[:4], streams, 3000, general=True)


def test_poisoned_shard_takes_one_ctx(ctxs):
    """a key decrease inside one stream (inside one shard, so the host cuts do not see it): the
    shard's verdict sends the call to skv_compact on ctxs[0], whose outcome is the oracle's"""
    rng = random.Random(19)
    streams = _streams(rng, 6, 3000, 12000)
    keys = [f"k{i:011d}" for i in sorted(rng.sample(range(12000), 3000))]
    keys[1700], keys[1701] = keys[1701], keys[1700]
    streams[2] = (3, [_fixed_run(keys, 40, 2)])
    _check(ctxs[:4], streams, 2500, split=False)


def test_corrupt_run_error_text(ctxs):
    """a truncated run: the error is the reference's, reported on ctxs[0]"""
    rng = random.Random(23)
    streams = _streams(rng, 4, 2000, 8000)
    streams[1] = (2, [streams[1][1][0][:-7]])
    exp, got = _both(ctxs[:3], streams, 4000)
    assert exp == got and exp[0] == "err", _diff(exp, got)


def test_one_ctx_is_compact(ctxs):
    rng = random.Random(29)
    streams = _streams(rng, 4, 2000, 8000)
    exp, got = _both(ctxs[:1], streams, 4000)
    assert exp == got, _diff(exp, got)


def test_repeated_ctx_is_rejected(ctxs):
    rng = random.Random(31)
    streams = _streams(rng, 2, 500, 2000)
    with pytest.raises(_abi.RunError) as ei:
        compact_split([ctxs[0], ctxs[1], ctxs[0]], streams, 4000)
    assert ei.value.code == _abi.SKV_E_INVALID_ARG


def test_result_kept_and_freed(ctxs):
    """keep=True: the result's pinned bytes (ctxs[0]'s pool) outlive the call and read back equal"""
    rng = random.Random(37)
    streams = _streams(rng, 5, 3000, 9000)
    exp = pyoracle.compact(streams, 3000, 0)
    res = compact_split(ctxs[:4], streams, 3000, keep=True)
    try:
        data = bytes(res.host_bytes())
        assert data == b"".join(r.data for r in exp)
        assert res.n_runs == len(exp)
    finally:
        res.free()


def test_tiny_call(ctxs):
    """fewer records than the fused split's parts need (64 per part): the general split"""
    rng = random.Random(41)
    _check(ctxs[:4], _streams(rng, 2, 50, 400), 2000, general=True)


# ---- variable-length records: build_runs' split carried from part to part ----------------------


@pytest.mark.parametrize("G", [2, 3, 8])
@pytest.mark.parametrize("max_size", [4096, 1000, 64 * 1024, 1 << 62, (1 << 64) - 1])
@pytest.mark.parametrize("flags", [0, _abi.SKV_DROP_TOMBSTONES], ids=["flags0", "drop"])
def test_general_split_matches_oracle(ctxs, G, max_size, flags):
    """config 3's shape (8-128 B keys, 10 % Deletes): runs continue across part edges"""
    streams = gen.config3(seed=900 + G, n_streams=12, run_bytes=96 * 1024)
    _check(ctxs[:G], streams, max_size, flags, general=True)


@pytest.mark.parametrize("parts", [2, 5])
def test_general_split_parts_per_ctx(ctxs, parts):
    streams = gen.config3(seed=77, n_streams=8, run_bytes=128 * 1024)
    _check(ctxs[:3], streams, 5000, 0, general=True, parts=parts)


@pytest.mark.parametrize("max_size", [1, 200, 400])
def test_general_split_runs_of_one_record(ctxs, max_size):
    """max below most records: nearly every record its own run, carried runs already over max"""
    streams = gen.config3(seed=31, n_streams=6, run_bytes=32 * 1024)
    _check(ctxs[:4], streams, max_size, 0, general=True)


def test_general_split_part_of_only_tombstones(ctxs):
    """a key range holding only Deletes: with the filter, a part with no survivors passes the
    carried run on unchanged"""
    rng = random.Random(8)
    streams = []
    for s in range(4):
        ids = sorted(rng.sample(range(40000), 3000))
        ops = [fmt.delete(f"k{i:06d}") if 10000 <= i < 30000 else fmt.put(f"k{i:06d}", b"x" * (i % 50))
               for i in ids]
        streams.append((s + 1, [fmt.encode_run(ops)]))
    _check(ctxs[:4], streams, 3000, _abi.SKV_DROP_TOMBSTONES, general=True, parts=3)


def test_general_split_member_runs(ctxs):
    """an L0 shape with variable records: a stream of many ascending member runs"""
    rng = random.Random(12)
    ids = sorted(rng.sample(range(300000), 30000))
    members = [fmt.encode_run([fmt.put(f"key{i:07d}", b"v" * (i % 97)) for i in ids[j:j + 1500]])
               for j in range(0, len(ids), 1500)]
    streams = [(0, members)] + [
        (s + 1, [fmt.encode_run([fmt.put(f"key{i:07d}", b"w" * (i % 31)) for i in sorted(rng.sample(range(300000), 4000))])])
        for s in range(3)]
    _check(ctxs[:4], streams, 8000, general=True)


def test_general_split_unsorted_stream(ctxs):
    """a key decrease inside a part: the part's decode check stops the split, skv_compact on
    ctxs[0] gives the oracle's outcome"""
    streams = gen.config3(seed=5, n_streams=6, run_bytes=48 * 1024)
    rng = random.Random(6)
    ids = sorted(rng.sample(range(100000), 2000))
    ops = [fmt.put(f"key{i:07d}", b"z" * (i % 40)) for i in ids]
    ops[900], ops[901] = ops[901], ops[900]
    streams[2] = (streams[2][0], [fmt.encode_run(ops)])
    _check(ctxs[:4], streams, 4096, split=False)


@pytest.mark.parametrize("G", [2, 4])
@pytest.mark.parametrize("max_size", [1 << 62, 16 * 1024])
def test_wal_flush_split(ctxs, G, max_size):
    """a WAL flush (SKV_SPLIT_BY_TABLE, 3,000 runs over 64 tables): parts cut at table prefixes hold
    whole tables, so nothing is carried. At 16 KiB every table breaks the one-run rule: the exact WAL
    stage, which a part does not run, so the call is skv_compact's (dropped_tables compared too)"""
    streams = [(s + 1, [gen.wal_run(700 + s).tobytes()]) for s in range(3000)]
    one_run = max_size == 1 << 62
    _check(ctxs[:G], streams, max_size, _abi.SKV_SPLIT_BY_TABLE, split=False, general=one_run)


@pytest.mark.parametrize("seed", list(range(40)) + [1077, 1203, 1238])
def test_split_random_shapes(ctxs, seed):
    """random calls: G, parts per ctx, record sizes (fixed or variable, with or without Deletes),
    fan-in, member runs, max_run_size and flags drawn per seed; either split, same bytes as the
    oracle. Seeds 1077 / 1203 / 1238 (tools/r05/split_fuzz.py): a part whose first pass was rerun
    (a deferred verification) after its split had already handed the next part a carried run from
    that first pass -- carried runs are now handed on only once a part's result is final"""
    rng = random.Random(10007 * seed + 3)
    G = rng.choice([2, 3, 4, 5, 8])
    parts = rng.choice([1, 1, 2, 3])
    flags = rng.choice([0, 0, _abi.SKV_DROP_TOMBSTONES])
    fixed = rng.random() < 0.4
    vlen = rng.choice([0, 8, 40, 200])
    space = rng.choice([2000, 20000, 200000])
    streams = []
    for s in range(rng.randint(1, 12)):
        n = rng.randint(0, 3000)
        ids = sorted(rng.sample(range(space), min(n, space)))
        if not ids:
            continue
        n_members = rng.choice([1, 1, 1, 3])
        cuts = sorted(rng.sample(range(1, len(ids)), min(n_members - 1, len(ids) - 1))) if len(ids) > 1 else []
        bounds = [0] + cuts + [len(ids)]
        members = []
        for a, b in zip(bounds, bounds[1:]):
            ops = []
            for i in ids[a:b]:
                key = f"k{i:09d}" if fixed else f"k{i:09d}" + "x" * (i % 13)  # (order-preserving)
                if not fixed and rng.random() < 0.1:
                    ops.append(fmt.delete(key))
                else:
                    ops.append(fmt.put(key, bytes([i & 0xFF]) * (vlen if fixed else (i * 7) % (vlen + 1))))
            members.append(fmt.encode_run(ops))
        streams.append((s + 1, members))
    if not streams:
        return
    max_size = rng.choice([1, 100, 1000, 4096, 1 << 20, 1 << 62])
    os.environ["SKV_SPLIT_PARTS"] = str(parts)
    try:
        exp, got = _both(ctxs[:G], streams, max_size, flags)
    finally:
        os.environ.pop("SKV_SPLIT_PARTS", None)
    assert exp == got, _diff(exp, got)
