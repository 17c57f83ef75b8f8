"""ScanFromRun on the device (skv_scan_runs: cache_service.rs:97-151 over read_run_iter,
runs.rs:400-510) against the reference's own scan tests (cache_service.rs:273-391,
tests/golden/kat.json kind "scan") and against the CPU restatement (oracle/ skvo_scan_runs), bit-exact:
response bytes, StatsV1, status code and error text."""
import json
import os
import random

import pytest

from skv import _abi
from skv import format as fmt
from skv.api import Compactor

import pyoracle
from test_scan_oracle import KATS, _ops, norm_oracle, scan_case
from knobs import knob, knob_get  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    torch = pytest.importorskip("torch")
    torch.cuda.init()
    c = Compactor(0)
    yield c
    c.close()


def norm_dev(dev, runs, start, mx):
    try:
        out = dev.scan_runs(runs, start, mx)
        assert len(out) <= 1
        return ("ok", [(r.data, r.stats.min_key, r.stats.max_key, r.stats.put_count, r.stats.delete_count)
                       for r in out])
    except _abi.RunError as e:
        return ("err", e.code, e.message)


@pytest.mark.parametrize("kat", KATS, ids=lambda k: k["name"])
def test_scan_kat_on_device(dev, kat):
    runs = [fmt.encode_run(_ops(ops)) for ops in kat["runs"]]
    start = bytes.fromhex(kat["start"])
    exp = kat["expect"]
    if "error" in exp:
        with pytest.raises(_abi.RunError) as ei:
            dev.scan_runs(runs, start, kat["max"])
        assert (ei.value.code, ei.value.message) == (_abi.SKV_E_INVALID_ARG, exp["message"])
        return
    out = dev.scan_runs(runs, start, kat["max"])
    assert [r.data for r in out] == [fmt.encode_run(_ops(exp["ops"]))]


@pytest.mark.parametrize("block", range(6))
def test_scan_random_cases_match_oracle(dev, block):
    """100 generated requests per block: corrupt / truncated / unsorted runs, start keys, cut-offs"""
    for seed in range(block * 100, block * 100 + 100):
        runs, start, mx = scan_case(seed)
        exp = norm_oracle(pyoracle, runs, start, mx)
        got = norm_dev(dev, runs, start, mx)
        assert got == exp, f"seed {seed}: {got} vs {exp}"


def _big_runs(rng, n_runs, n_rec, space, del_frac=0.1, vmax=40):
    runs = []
    for i in range(n_runs):
        ids = sorted(rng.sample(range(space), n_rec))
        ops = []
        for k in ids:
            key = f"user{k:08d}" + ("x" * (k % 23))  # keys past the 16-byte prefix too
            if rng.random() < del_frac:
                ops.append(fmt.delete(key))
            else:
                ops.append(fmt.put(key, bytes([i & 0xFF]) * rng.randint(0, vmax)))
        runs.append(fmt.encode_run(ops))
    return runs


@pytest.mark.parametrize("mx", [1, 7, 100, 10000])
@pytest.mark.parametrize("start", [b"", b"user00030000", b"user00059999xxx", b"zzz"])
def test_scan_many_records(dev, mx, start):
    rng = random.Random(mx * 7 + len(start))
    runs = _big_runs(rng, 12, 4000, 60000)
    assert norm_dev(dev, runs, start, mx) == norm_oracle(pyoracle, runs, start, mx)


def test_scan_unsorted_and_corrupt_large(dev):
    """heap pop order at size: a run with decreases, a descending run, a run cut inside a
    value-length field"""
    rng = random.Random(5)
    runs = _big_runs(rng, 6, 3000, 20000)
    ids = sorted(rng.sample(range(20000), 3000))
    for _ in range(40):  # adjacent swaps: decreases inside the run
        i = rng.randrange(len(ids) - 1)
        ids[i], ids[i + 1] = ids[i + 1], ids[i]
    runs[2] = fmt.encode_run([fmt.put(f"user{k:08d}", b"s") for k in ids])
    runs.append(fmt.encode_run(list(reversed([(True, f"k{i:05d}".encode(), b"v") for i in range(500)]))))
    runs[4] = runs[4][: len(runs[4]) // 2] + b"\x01\x00\x00\x00\x02ab\x00"
    for mx in (1, 50, 2000, 10000):
        for start in (b"", b"k00100", b"user00010000"):
            assert norm_dev(dev, runs, start, mx) == norm_oracle(pyoracle, runs, start, mx), (mx, start)


def test_scan_record_sort_path(dev):
    """SKV_SORT=1 sends the merge through the record sort (the > 768-run path): same responses"""
    rng = random.Random(9)
    runs = _big_runs(rng, 5, 2000, 8000)
    runs.append(fmt.encode_run(list(reversed([(True, f"user{i:08d}".encode(), b"q") for i in range(300)]))))
    old = knob_get("SKV_SORT")
    knob("SKV_SORT", "1")
    try:
        for mx in (3, 500, 10000):
            for start in (b"", b"user00004000"):
                assert norm_dev(dev, runs, start, mx) == norm_oracle(pyoracle, runs, start, mx), (mx, start)
    finally:
        if old is None:
            knob("SKV_SORT", None)
        else:
            knob("SKV_SORT", old)


def test_scan_more_runs_than_the_splitter_merge_takes(dev):
    """1,000 runs (record sort by fan-in) with a few corrupt ones"""
    rng = random.Random(13)
    runs = _big_runs(rng, 1000, 20, 5000, vmax=8)
    for i in (17, 501, 998):
        runs[i] = runs[i] + b"\x02\x00\x00"
    for mx in (1, 100, 10000):
        assert norm_dev(dev, runs, b"user00001000", mx) == norm_oracle(pyoracle, runs, b"user00001000", mx)
