"""ScanFromRun (cache_service.rs:97-151) over read_run_iter (runs.rs:400-510) in the CPU restatement
(oracle/skv_oracle.c skvo_scan_runs) — pinned by the reference's own scan tests
(cache_service.rs:273-391, tests/golden/kat.json kind "scan") and by the independent Python
restatement (tests/pyref.py scan) on generated inputs: corrupt and truncated runs (RunIterator's
own error texts), unsorted runs (heap pop order), start keys inside and between runs, and
max_results cut-offs that hide or reveal a later merge error."""
import json
import os
import random

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import pyref
from skv import format as fmt
from test_oracle_vs_pyref import _run

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KATS = [k for k in json.load(open(os.path.join(GOLDEN, "kat.json"))) if k["kind"] == "scan"]
STARTS = [b"", b"a", b"ab", b"b", b"b0", b"c", b"p" * 20, b"zz", b"\xc3\xa9", b"zzz"]


def _ops(lst):
    return [(o["put"], bytes.fromhex(o["key"]), bytes.fromhex(o["val"]) if o["put"] else None) for o in lst]


def scan_case(seed: int):
    """(runs, start key, max_results) for one generated scan request."""
    r = random.Random(seed)
    sorted_ok = r.random() < 0.85
    runs = [_run(r, False, sorted_ok) for _ in range(r.randint(0, 6))]
    for i in range(len(runs)):  # truncations inside a length field: RunIterator's own texts
        if r.random() < 0.05 and len(runs[i]) > 3:
            runs[i] = runs[i] + bytes([r.choice([1, 2])]) + b"\x00" * r.randint(0, 3)
        elif r.random() < 0.04 and len(runs[i]) > 1:
            runs[i] = runs[i] + b"\x01\x00\x00\x00\x01k" + b"\x00" * r.randint(0, 3)
    start = r.choice(STARTS)
    mx = r.choice([1, 1, 2, 3, 5, 8, 10000, 10000, 0, 10001])
    return runs, start, mx


def norm_oracle(oracle, runs, start, mx):
    try:
        out = oracle.scan_runs(runs, start, mx)
        assert len(out) <= 1
        return ("ok", [(r.data, r.stats.min_key, r.stats.max_key, r.stats.put_count, r.stats.delete_count)
                       for r in out])
    except Exception as e:
        return ("err", e.code, e.message)


def norm_pyref(runs, start, mx):
    try:
        items = pyref.scan(runs, start, mx)
    except pyref.Err as e:
        return ("err", e.code, e.msg)
    if not items:
        return ("ok", [])
    data = fmt.encode_run([(k == "put", key, v) for k, key, v in items])
    return ("ok", [(data, items[0][1].decode(), items[-1][1].decode(), sum(k == "put" for k, _, _ in items),
                    sum(k == "del" for k, _, _ in items))])


@pytest.mark.parametrize("kat", KATS, ids=lambda k: k["name"])
def test_scan_kat(kat, oracle):
    runs = [fmt.encode_run(_ops(ops)) for ops in kat["runs"]]
    start = bytes.fromhex(kat["start"])
    exp = kat["expect"]
    if "error" in exp:
        with pytest.raises(Exception) as ei:
            oracle.scan_runs(runs, start, kat["max"])
        assert ei.value.code == 6 and ei.value.message == exp["message"]
        return
    out = oracle.scan_runs(runs, start, kat["max"])
    assert [r.data for r in out] == [fmt.encode_run(_ops(exp["ops"]))]


@settings(max_examples=500, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.integers(min_value=0, max_value=2**32))
def test_scan_oracle_matches_pyref(oracle, seed):
    runs, start, mx = scan_case(seed)
    assert norm_oracle(oracle, runs, start, mx) == norm_pyref(runs, start, mx)


def test_iterator_error_texts(oracle):
    """RunIterator's two EOF checks are Format errors with their own text (runs.rs:428-430,
    :457-459) where read_run_stream raises Io — the scan reports them as the iterator does."""
    good = fmt.encode_run([fmt.put("k", b"v")])
    for tail, text in ((b"\x01\x00\x00", "Data format error: Incomplete key length data"),
                       (b"\x01\x00\x00\x00\x01z\x00\x00", "Data format error: Incomplete value length data"),
                       (b"\x01\x00\x00\x00\x05ab", "Data format error: Incomplete key data"),
                       (b"\x07\x00\x00\x00\x01z", "Data format error: Invalid marker byte: 7")):
        with pytest.raises(Exception) as ei:
            oracle.scan_runs([good + tail], b"", 10)
        assert (ei.value.code, ei.value.message) == (4, text)
        assert norm_pyref([good + tail], b"", 10) == ("err", 4, text)


def test_cutoff_hides_a_later_error(oracle):
    """The reader stops right after the max_results-th Put; a decode error the merge would raise
    after that is never seen (cache_service.rs:140-148)."""
    run = fmt.encode_run([fmt.put("a", b"1"), fmt.put("b", b"2")]) + b"\x01\x00"
    assert [r.stats.put_count for r in oracle.scan_runs([run], b"", 1)] == [1]
    assert [r.stats.put_count for r in oracle.scan_runs([run], b"", 2)] == [2]  # stops right after "b"
    with pytest.raises(Exception):
        oracle.scan_runs([run], b"", 3)  # the error follows "b"'s refill, before a 3rd Put
    # a start key past every good record: the error is the stream's first item
    with pytest.raises(Exception) as ei:
        oracle.scan_runs([run], b"b", 1)
    assert ei.value.message == "Data format error: Incomplete key length data"
