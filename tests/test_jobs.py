"""The job wrappers (skyvault-rs_amd/skv/jobs.py) against the reference jobs' semantics
(src/jobs/*.rs): stream assembly (16-run cap, L0 concatenated at SeqNo 0, level-L run at SeqNo 1
over the overlapping L+1 runs), the Delete filter at Level::max(), the WAL split, what is marked
compacted (ALL buffer / WAL runs, although only 16 are merged), the "No runs were generated"
internal error, and BASELINE config 1's plumbing (encode -> in-memory object store -> compact ->
put). CPU tests drive the job code with the oracle as the compactor; the gpu-marked tests run
the same jobs on the device path and require identical results. The quirks are pinned by
tests/golden/job_quirks.json (tests/golden/make_job_fixtures.py) so that a "fixed" behaviour is
never adopted silently.
"""
import json
import os

import pytest

from skv import _abi, gen, jobs
from skv import format as fmt

import pyoracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "job_quirks.json")


class OracleCompactor:
    """The oracle behind the same compact() signature as skv.api.Compactor (tests only)."""

    def __init__(self):
        self.calls = []

    def compact(self, streams, max_run_size, flags, with_info=False):
        self.calls.append(([(s, len(r)) for s, r in streams], max_run_size, flags))
        return pyoracle.compact(streams, max_run_size, flags, with_result=with_info)


class Recording:
    def __init__(self, inner):
        self.inner = inner
        self.calls = []

    def compact(self, streams, max_run_size, flags, with_info=False):
        self.calls.append(([(s, len(r)) for s, r in streams], max_run_size, flags))
        return self.inner.compact(streams, max_run_size, flags, with_info=with_info)


def _run(ops):
    return fmt.encode_run(ops)


def _meta(store, data, seq_hint=""):
    rid = jobs.new_run_id()
    store.put_run(rid, data)
    ops, _ = pyoracle.decode_run(data)
    keys = [o[1].decode() for o in ops]
    st = _abi.Stats(min(keys) if keys else "", max(keys) if keys else "", len(data),
                    sum(1 for o in ops if o[0]), sum(1 for o in ops if not o[0]))
    return jobs.RunMeta(rid, st)


def _buffer_table(store, n_buffer=20, n_l0=3):
    t = jobs.TableTree()
    for s in range(n_buffer):
        keys = sorted({f"k{(s * 7 + i) % 50:03d}" for i in range(5)})
        t.buffer[100 + s] = _meta(store, _run([fmt.put(k, b"b%d" % s) for k in keys]))
    t.tree[0] = {}
    for j in range(n_l0):
        m = _meta(store, _run([fmt.put(f"k{j * 20 + i:03d}", b"L0") for i in range(10)]))
        t.tree[0][m.stats.min_key] = m
    return t


def _jobs_outcome(compactor):
    """Every quirk case through the job code; a JSON-able summary (bytes by hex)."""
    out = {}
    store = jobs.MemoryObjectStore()
    t = _buffer_table(store)
    rec = Recording(compactor)
    compacted, new = jobs.table_buffer_compaction(rec, store, 7, t)
    out["buffer_20_plus_l0"] = {
        "streams": rec.calls[0][0], "flags": rec.calls[0][2], "max": rec.calls[0][1],
        "compacted": len(compacted), "all_buffer_and_l0_marked": compacted == [m.id for _, m in sorted(t.buffer.items())]
        + [m.id for _, m in sorted(t.tree[0].items())],
        "runs": [store.runs[r.id].hex() for r in new], "belongs_to": [list(r.belongs_to) for r in new]}
    # buffer runs holding no records: build_runs yields nothing -> JobError::Internal
    t2 = jobs.TableTree(buffer={1: _meta(store, b"\x01"), 2: _meta(store, b"\x01")})
    try:
        jobs.table_buffer_compaction(compactor, store, 8, t2)
        out["buffer_no_output"] = "ok"
    except jobs.JobError as e:
        out["buffer_no_output"] = [e.kind, str(e)]
    out["buffer_empty_table"] = list(jobs.table_buffer_compaction(compactor, store, 9, jobs.TableTree()))
    # tree compaction: level 5 -> 6 drops Deletes; overlap selection; level 6 is never compacted
    t3 = jobs.TableTree()
    lvl = _meta(store, _run([fmt.put("m10", b"new"), fmt.delete("m20"), fmt.put("m30", b"new")]))
    t3.tree[5] = {lvl.stats.min_key: lvl}
    t3.tree[6] = {}
    for keys in (["a00", "a05"], ["m05", "m15"], ["m25", "m40"], ["z00"]):
        m = _meta(store, _run([fmt.put(k, b"old") for k in keys]))
        t3.tree[6][m.stats.min_key] = m
    rec = Recording(compactor)
    compacted, new = jobs.table_tree_compaction(rec, store, 3, t3, 5)
    out["tree_5_to_6"] = {"streams": rec.calls[0][0], "flags": rec.calls[0][2], "compacted": len(compacted),
                          "runs": [store.runs[r.id].hex() for r in new],
                          "belongs_to": [list(r.belongs_to) for r in new]}
    out["tree_level_max"] = list(jobs.table_tree_compaction(compactor, store, 3, t3, 6))
    # an L+1 run containing the whole level-run range overlaps it too (:68-70)
    t3b = jobs.TableTree(tree={2: {lvl.stats.min_key: lvl}, 3: {}})
    for keys in (["a00"], ["l00", "n00"], ["z00"]):
        m = _meta(store, _run([fmt.put(k, b"old") for k in keys]))
        t3b.tree[3][m.stats.min_key] = m
    rec = Recording(compactor)
    compacted, new = jobs.table_tree_compaction(rec, store, 3, t3b, 2)
    out["tree_containing_run"] = {"streams": rec.calls[0][0], "flags": rec.calls[0][2],
                                  "runs": [store.runs[r.id].hex() for r in new]}
    # a level run whose merge leaves nothing (all Deletes at the max level): no error in tree jobs
    t4 = jobs.TableTree(tree={5: {}})
    d = _meta(store, _run([fmt.delete("q1"), fmt.delete("q2")]))
    t4.tree[5][d.stats.min_key] = d
    c4, n4 = jobs.table_tree_compaction(compactor, store, 4, t4, 5)
    out["tree_all_deleted"] = [len(c4), len(n4)]
    # WAL: 20 runs, 16 merged, all 20 compacted; a table whose build fails is dropped
    wal = {}
    for s in range(20):
        wal[s + 1] = _meta(store, _run([fmt.put(f"{t}.{s:03d}", b"w") for t in (1, 2, 7)]))
    rec = Recording(compactor)
    compacted, table_runs = jobs.wal_compaction(rec, store, wal)
    out["wal_20"] = {"streams": rec.calls[0][0], "flags": rec.calls[0][2], "compacted": len(compacted),
                     "tables": [t for _, t, _ in table_runs], "runs": [store.runs[r].hex() for r, _, _ in table_runs]}
    bad = {1: _meta(store, _run([fmt.put("1.a", b"x"), fmt.put("nodot", b"y")]))}
    try:
        jobs.wal_compaction(compactor, store, bad)
        out["wal_bad_key"] = "ok"
    except jobs.JobError as e:
        out["wal_bad_key"] = [e.kind, str(e)]
    corrupt = {1: _meta(store, _run([fmt.put("1.a", b"x"), fmt.put("2.b", b"y")])[:-1])}
    try:
        jobs.wal_compaction(compactor, store, corrupt)
        out["wal_corrupt"] = "ok"
    except jobs.JobError as e:
        out["wal_corrupt"] = [e.kind, str(e)]
    out["wal_due"] = [jobs.wal_compactor_due(wal), jobs.wal_compactor_due({i: wal[1] for i in range(25)})]
    # BASELINE config 1: 2 x ~1 MiB runs through the in-memory store and a buffer compaction
    t5 = jobs.TableTree()
    for seq, runs in gen.config1():
        t5.buffer[seq] = _meta(store, runs[0])
    compacted, new = jobs.table_buffer_compaction(compactor, store, 11, t5)
    import hashlib

    out["config1"] = {"compacted": len(compacted), "runs": len(new),
                      "sha256": hashlib.sha256(b"".join(store.runs[r.id] for r in new)).hexdigest(),
                      "sizes": [r.stats.size_bytes for r in new]}
    return out


def test_job_quirks_match_fixture():
    exp = json.load(open(GOLDEN))
    got = json.loads(json.dumps(_jobs_outcome(OracleCompactor())))
    assert got == exp


def test_job_quirks_direct():
    """The quirks themselves, spelled out (independently of the fixture)."""
    o = _jobs_outcome(OracleCompactor())
    b = o["buffer_20_plus_l0"]
    assert [s for s, _ in b["streams"]] == list(range(100, 116)) + [0]  # oldest 16 + L0 at SeqNo 0
    assert b["streams"][-1][1] == 3 and b["compacted"] == 23 and b["all_buffer_and_l0_marked"]
    assert o["buffer_no_output"] == ["Internal", "Internal error: No runs were generated during compaction"]
    assert o["buffer_empty_table"] == [[], []]
    assert o["tree_5_to_6"]["flags"] == _abi.SKV_DROP_TOMBSTONES
    assert [s for s, _ in o["tree_5_to_6"]["streams"]] == [1, 0]
    assert o["tree_5_to_6"]["streams"][1][1] == 2  # m05-m15 and m25-m40 overlap m10..m30
    assert o["tree_containing_run"]["streams"] == [(1, 1), (0, 1)] and o["tree_containing_run"]["flags"] == 0
    assert o["tree_level_max"] == [[], []]
    assert o["tree_all_deleted"] == [1, 0]
    assert o["wal_20"]["compacted"] == 20 and len(o["wal_20"]["streams"]) == 16
    assert o["wal_20"]["tables"] == [1, 2, 7]
    assert o["wal_bad_key"][0] == "InvalidInput"
    assert o["wal_corrupt"][0] == "Run"
    assert o["wal_due"] == [False, True]


@pytest.mark.gpu
def test_job_quirks_on_device():
    torch = pytest.importorskip("torch")
    torch.cuda.init()
    from skv.api import Compactor

    c = Compactor(0)
    try:
        got = json.loads(json.dumps(_jobs_outcome(c)))
    finally:
        c.close()
    assert got == json.load(open(GOLDEN))
