"""The reference's own known-answer tests (tests/golden/kat.json) fed straight through the HIP
path (libskv.so, skv_compact) — each result is compared with the KAT's expected bytes and
StatsV1 directly, not with the oracle.

How a KAT maps onto the compaction boundary (skv.h: read_run_stream -> k_way::merge -> build_runs):
- build_runs KATs (runs.rs:775-920): the KAT's ops, encoded as ONE input run of ONE stream, are
  what build_runs sees after decode and a one-stream merge (the merge of one sorted stream is the
  stream itself, k_way.rs:144-172), so skv_compact(max) must give the KAT's runs byte for byte.
  test_create_run_with_duplicates: the merge drops a key equal to the last one emitted
  (k_way.rs:146-151) before build_runs can see it, so the compaction gives the first op; the
  build_runs order error of that test is reached through a strict decrease in the stream.
- merge KATs (k_way.rs:42-107, :186-226; cache_service.rs:349-391): each stream's ops as one run
  at the KAT's SeqNo; skv_compact with an unbounded max gives one run holding exactly the KAT's
  expected op sequence.
- test_create_multiple_runs_due_to_size (runs.rs:914-1000): 52 records of 1,048,576 B at max 2 MiB
  -> 52 runs of 1,048,577 B.
"""
import json
import os

import pytest

from skv import _abi
from skv import format as fmt
from skv.api import Compactor

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KATS = json.load(open(os.path.join(GOLDEN, "kat.json")))
KAT_BY_NAME = {k["name"]: k for k in KATS}
UNBOUNDED = 1 << 62


@pytest.fixture(scope="module")
def dev():
    torch = pytest.importorskip("torch")
    torch.cuda.init()
    c = Compactor(0)
    yield c
    c.close()


def _ops(lst):
    return [(o["put"], bytes.fromhex(o["key"]), bytes.fromhex(o["val"]) if o["put"] else None) for o in lst]


def _check_runs(runs, exp_runs):
    assert len(runs) == len(exp_runs)
    for r, e in zip(runs, exp_runs):
        assert r.data.hex() == e["hex"]
        assert r.data[0] == 1
        assert (r.stats.min_key, r.stats.max_key) == (e["min_key"], e["max_key"])
        assert r.stats.size_bytes == e["size_bytes"] == len(r.data)
        assert (r.stats.put_count, r.stats.delete_count) == (e["put_count"], e["delete_count"])


@pytest.mark.parametrize("kat", [k for k in KATS if k["kind"] == "build_runs"], ids=lambda k: k["name"])
def test_build_runs_kat_on_device(dev, kat):
    ops = _ops(kat["ops"])
    exp = kat["expect"]
    runs = dev.compact([(1, [fmt.encode_run(ops)])], kat["max"], 0)
    if "error" in exp:
        # duplicates never reach build_runs through the merge: the first op of the key survives
        first = []
        for op in ops:
            if not first or first[-1][1] != op[1]:
                first.append(op)
        assert [r.data for r in runs] == [fmt.encode_run(first)]
        # build_runs' own order error (runs.rs:190-198), reached through a strict decrease
        with pytest.raises(_abi.RunError) as ei:
            dev.compact([(1, [fmt.encode_run([ops[0], (True, b"0" + ops[0][1][:0], b"x")])])], kat["max"], 0)
        assert (ei.value.code, ei.value.message) == (_abi.SKV_E_FORMAT, exp["message"])
        return
    if "same_as" in exp:
        other = KAT_BY_NAME[exp["same_as"]]
        _check_runs(runs, other["expect"]["runs"])
        return
    if "runs" in exp:
        _check_runs(runs, exp["runs"])
    if "n_runs" in exp:
        assert len(runs) == exp["n_runs"]
        # the round trip: the run holds exactly the KAT's ops, and searching it gives the KAT's
        # answers (runs::search_run, runs.rs:285-398, on the device)
        assert [r.data for r in runs] == [fmt.encode_run(ops)]
        keys = list(exp.get("search", {}))
        if keys:
            got = dev.search_run(runs[0].data, [k.encode() for k in keys])
            for k, g in zip(keys, got):
                kind, val = exp["search"][k]
                assert g == (kind, bytes.fromhex(val) if val is not None else None)


def test_multiple_runs_due_to_size_on_device(dev):
    kat = KAT_BY_NAME["test_create_multiple_runs_due_to_size"]
    g = kat["gen"]
    ops = []
    for i in range(g["count"]):
        key = (g["key_fmt"] % i).encode()
        ops.append((True, key, bytes((i * 7 + j) & 0xFF for j in range(g["record_size"] - (1 + 4 + len(key) + 4)))))
    runs = dev.compact([(1, [fmt.encode_run(ops)])], kat["max"], 0)
    assert len(runs) == kat["expect"]["n_runs"]
    for i, r in enumerate(runs):
        assert r.stats.size_bytes == kat["expect"]["size_bytes_each"] == len(r.data)
        assert r.stats.min_key == r.stats.max_key == g["key_fmt"] % i
        assert r.data == fmt.encode_run([ops[i]])


@pytest.mark.parametrize("kat", [k for k in KATS if k["kind"] == "merge"], ids=lambda k: k["name"])
def test_merge_kat_on_device(dev, kat):
    streams = [(s, [fmt.encode_run(_ops(ops))]) for s, ops in kat["streams"]]
    exp_ops = _ops(kat["expect"]["ops"])
    runs = dev.compact(streams, UNBOUNDED, 0)
    assert [r.data for r in runs] == [fmt.encode_run(exp_ops)]
    r = runs[0]
    assert (r.stats.min_key.encode(), r.stats.max_key.encode()) == (exp_ops[0][1], exp_ops[-1][1])
    assert r.stats.put_count == sum(1 for o in exp_ops if o[0])
    assert r.stats.delete_count == sum(1 for o in exp_ops if not o[0])
    # the same streams in the other vector order: the merge order depends on SeqNo only
    runs = dev.compact(list(reversed(streams)), UNBOUNDED, 0)
    assert [r.data for r in runs] == [fmt.encode_run(exp_ops)]


@pytest.mark.parametrize("kat", [k for k in KATS if k["kind"] == "decode"], ids=lambda k: k["name"])
def test_decode_kat_on_device(dev, kat):
    """Hand-derived decode cases (runs.rs:517-628): one stream of the KAT's run. A decode error
    surfaces with the reference's text; a clean run round-trips."""
    run = bytes.fromhex(kat["hex"])
    exp = kat["expect"]
    if exp["error"] is not None:
        with pytest.raises(_abi.RunError) as ei:
            dev.compact([(1, [run])], UNBOUNDED, 0)
        assert ei.value.message == exp["message"]
        return
    runs = dev.compact([(1, [run])], UNBOUNDED, 0)
    assert [r.data for r in runs] == ([run] if exp["n_ops"] else [])
