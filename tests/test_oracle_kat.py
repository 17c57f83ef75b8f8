"""Pins the CPU restatement (oracle/) to the reference's own known-answer tests
(tests/golden/kat.json, transcribed from runs.rs / k_way.rs / cache_service.rs tests) and to
the generated compaction fixtures (tests/golden/compact_cases.json)."""
import hashlib
import json
import os

import pytest

from skv import format as fmt

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KATS = json.load(open(os.path.join(GOLDEN, "kat.json")))
CASES = json.load(open(os.path.join(GOLDEN, "compact_cases.json")))
KAT_BY_NAME = {k["name"]: k for k in KATS}


def _ops(lst):
    return [(o["put"], bytes.fromhex(o["key"]), bytes.fromhex(o["val"]) if o["put"] else None) for o in lst]


def _search(run: bytes, key: bytes, oracle):
    """runs::search_run semantics (runs.rs:285-398) over the oracle's decode of one run."""
    ops, err = oracle.decode_run(run)
    assert err is None
    for is_put, k, v in ops:
        if k == key:
            return ("found", v.hex()) if is_put else ("tombstone", None)
        if k > key:
            return ("not_found", None)
    return ("not_found", None)


@pytest.mark.parametrize("kat", [k for k in KATS if k["kind"] == "build_runs"], ids=lambda k: k["name"])
def test_build_runs_kat(kat, oracle):
    ops = _ops(kat["ops"])
    exp = kat["expect"]
    if "error" in exp:
        with pytest.raises(Exception) as ei:
            oracle.build_runs(ops, kat["max"])
        assert ei.value.kind == exp["error"]
        assert ei.value.message == exp["message"]
        return
    runs = oracle.build_runs(ops, kat["max"])
    if "same_as" in exp:
        other = KAT_BY_NAME[exp["same_as"]]
        assert [r.data for r in runs] == [r.data for r in oracle.build_runs(_ops(other["ops"]), other["max"])]
        return
    if "runs" in exp:
        assert len(runs) == len(exp["runs"])
        for r, e in zip(runs, exp["runs"]):
            assert r.data.hex() == e["hex"]
            assert r.data[0] == 1
            assert r.stats.min_key == e["min_key"] and r.stats.max_key == e["max_key"]
            assert r.stats.size_bytes == e["size_bytes"] == len(r.data)
            assert (r.stats.put_count, r.stats.delete_count) == (e["put_count"], e["delete_count"])
    if "n_runs" in exp:
        assert len(runs) == exp["n_runs"]
    for key, (kind, val) in exp.get("search", {}).items():
        assert _search(runs[0].data, key.encode(), oracle) == (kind, val)


def test_multiple_runs_due_to_size(oracle):
    kat = KAT_BY_NAME["test_create_multiple_runs_due_to_size"]
    g = kat["gen"]
    ops = []
    for i in range(g["count"]):
        key = (g["key_fmt"] % i).encode()
        overhead = 1 + 4 + len(key) + 4
        ops.append((True, key, bytes(g["record_size"] - overhead)))
    runs = oracle.build_runs(ops, kat["max"])
    assert len(runs) == kat["expect"]["n_runs"]
    prev = None
    for i, r in enumerate(runs):
        assert r.stats.size_bytes == kat["expect"]["size_bytes_each"] == len(r.data)
        assert r.stats.size_bytes <= kat["max"]
        assert r.stats.min_key == r.stats.max_key == g["key_fmt"] % i
        if prev is not None:
            assert r.stats.min_key > prev
        prev = r.stats.max_key


@pytest.mark.parametrize("kat", [k for k in KATS if k["kind"] == "merge"], ids=lambda k: k["name"])
def test_merge_kat(kat, oracle):
    streams = [(s, _ops(ops)) for s, ops in kat["streams"]]
    out, err = oracle.merge_ops(streams)
    assert err is None
    assert out == _ops(kat["expect"]["ops"])


@pytest.mark.parametrize("kat", [k for k in KATS if k["kind"] == "decode"], ids=lambda k: k["name"])
def test_decode_kat(kat, oracle):
    ops, err = oracle.decode_run(bytes.fromhex(kat["hex"]))
    exp = kat["expect"]
    assert len(ops) == exp["n_ops"]
    if exp["error"] is None:
        assert err is None
    else:
        assert err is not None and err.kind == exp["error"] and err.message == exp["message"]


def test_golden_run_bytes_match_format_writer():
    """The 39-byte golden run equals what the host format writer produces for the same ops."""
    kat = KAT_BY_NAME["test_create_run_simple"]
    assert fmt.encode_run(_ops(kat["ops"])).hex() == kat["expect"]["runs"][0]["hex"]


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_compact_fixture(case, oracle):
    streams = [(s, [bytes.fromhex(r) for r in runs]) for s, runs in case["streams"]]
    exp = case["expect"]
    if "error_code" in exp:
        with pytest.raises(Exception) as ei:
            oracle.compact(streams, case["max"], case["flags"])
        assert ei.value.code == exp["error_code"] and ei.value.message == exp["message"]
        return
    runs, info = oracle.compact(streams, case["max"], case["flags"], with_result=True)
    assert [r.data.hex() for r in runs] == [e["hex"] for e in exp["runs"]]
    assert [r.table_id for r in runs] == [e["table_id"] for e in exp["runs"]]
    assert [(r.stats.size_bytes, r.stats.put_count, r.stats.delete_count) for r in runs] == \
        [(e["size_bytes"], e["put_count"], e["delete_count"]) for e in exp["runs"]]
    assert [r.stats.min_key.encode().hex() for r in runs] == [e["min_key"] for e in exp["runs"]]
    assert [r.stats.max_key.encode().hex() for r in runs] == [e["max_key"] for e in exp["runs"]]
    assert info["dropped_tables"] == exp["dropped_tables"]
    assert hashlib.sha256(b"".join(r.data for r in runs)).hexdigest() == case["sha256"]
