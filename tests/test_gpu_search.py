"""GPU parity of the batched run lookup (skv_search_run): runs::search_run (runs.rs:285-398) for
many keys at once, against a literal restatement (oracle/pyoracle.search_run), including every
panic class and the reference's own search KATs (runs.rs:823-883, tests/golden/kat.json)."""
import random

import pytest

from skv import format as fmt
from skv.api import Compactor

import pyoracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    torch = pytest.importorskip("torch")
    torch.cuda.init()
    c = Compactor(0, profiling=True)
    yield c
    c.close()


def _check(dev, run, keys):
    got = dev.search_run(run, keys)
    exp = [pyoracle.search_run(run, k) for k in keys]
    bad = [(k, e, g) for k, e, g in zip(keys, exp, got) if e != g]
    assert not bad, bad[:5]
    return got


def _sorted_run(r, n, vmax=20, deletes=0.2, dup=0.0):
    keys = sorted({f"key{r.randrange(10 * n + 1):07d}".encode() + b"~" * r.randint(0, 20) for _ in range(n)})
    ops = []
    for k in keys:
        ops.append(fmt.delete(k) if r.random() < deletes else fmt.put(k, r.randbytes(r.randint(0, vmax))))
        if r.random() < dup:
            ops.append(fmt.put(k, b"dup"))
    return fmt.encode_run(ops), keys


def test_search_kats(dev):
    """The reference's own search tests (runs.rs:823-884), expected outcomes transcribed."""
    run = fmt.encode_run([fmt.put("apple", b"red"), fmt.put("banana", b"yellow"), fmt.put("cherry", b"red")])
    assert dev.search_run(run, [b"banana", b"apple", b"cherry"]) == \
        [("found", b"yellow"), ("found", b"red"), ("found", b"red")]           # test_search_run_found
    run = fmt.encode_run([fmt.put("apple", b"red"), fmt.delete("banana"), fmt.put("cherry", b"red")])
    assert dev.search_run(run, [b"banana", b"apple"]) == [("tombstone", None), ("found", b"red")]
    run = fmt.encode_run([fmt.put("banana", b"yellow"), fmt.put("date", b"brown")])
    assert dev.search_run(run, [b"apple", b"cherry", b"elderberry"]) == [("not_found", None)] * 3
    assert dev.search_run(b"", [b"any"]) == [("panic", "Empty run data")]    # test_search_run_empty_data
    assert dev.search_run(bytes([2, 0]), [b"any"]) == [("panic", "Unsupported version: 2")]


@pytest.mark.parametrize("n", [1, 7, 300, 20000])
def test_search_clean_sorted_runs(dev, n):
    r = random.Random(n)
    run, keys = _sorted_run(r, n)
    some = keys if len(keys) <= 300 else r.sample(keys, 300)  # the restatement scans in Python
    queries = list(some) + [k + b"\x00" for k in some[:50]] + [k[:-1] for k in some[:50]] + \
        [f"key{r.randrange(10 * n + 1):07d}".encode() for _ in range(200)] + [b"", b"\xff" * 3, b"a", b"zzzz"]
    _check(dev, run, queries)


def test_search_duplicates_and_unsorted(dev):
    r = random.Random(4)
    run, keys = _sorted_run(r, 400, dup=0.3)   # equal neighbours: first one wins
    _check(dev, run, keys + [b"nope"])
    ops = [fmt.put(f"k{i:03d}", bytes([i & 255])) for i in r.sample(range(300), 300)]  # unsorted: scan semantics
    _check(dev, fmt.encode_run(ops), [f"k{i:03d}".encode() for i in range(0, 320, 3)])


def test_search_panics(dev):
    r = random.Random(8)
    run, keys = _sorted_run(r, 200, vmax=8)
    qs = keys[::7] + [b"", b"zzz", keys[-1] + b"!"]
    cases = [b"", b"\x02" + run[1:], run[:-1], run[: len(run) // 2], run[:1], run[:3], run + b"\x05",
             run + b"\x01\x00\x00", run + b"\x01\x00\x00\x00\x09ab", run + b"\x01\x00\x00\x00\x03zzz\x00\x00",
             run + b"\x01\x00\x00\x00\x03zzz\x00\x00\x00\x09ab"]
    bad = bytearray(run)
    bad[len(run) // 3] = 0x09  # a marker/length byte in the middle
    cases.append(bytes(bad))
    bad2 = bytearray(run)
    bad2[1 + 5] = 0xFF  # invalid UTF-8 inside the first key: search_run does not check it
    cases.append(bytes(bad2))
    for c in cases:
        _check(dev, c, qs)


def test_run_index_many_batches(dev):
    """skv_run_index_*: the run staged and parsed once, then several lookup batches, each equal to
    skv_search_run and to the restatement — clean runs (binary search), unsorted / duplicate /
    corrupt runs (the scan) and the panic-only runs; two indexes alive on one ctx."""
    r = random.Random(12)
    runs = []
    run, keys = _sorted_run(r, 3000)
    runs.append((run, keys))
    run2, keys2 = _sorted_run(r, 500, dup=0.3)
    runs.append((run2, keys2))
    ops = [fmt.put(f"k{i:03d}", bytes([i & 255])) for i in r.sample(range(300), 300)]
    runs.append((fmt.encode_run(ops), [f"k{i:03d}".encode() for i in range(0, 320, 3)]))
    runs.append((run[: len(run) // 2], keys[::5]))
    runs.append((b"", [b"a"]))
    runs.append((b"\x03" + run[1:], [b"a"]))
    idx = [(dev.run_index(rb), rb, ks) for rb, ks in runs]
    try:
        for batch in range(3):
            for ix, rb, ks in idx:
                q = [k for k in ks if r.random() < 0.5][:200] + [b"zz%d" % batch, b""]
                exp = [pyoracle.search_run(rb, k) for k in q]
                assert ix.search(q) == exp
                assert dev.search_run(rb, q) == exp
    finally:
        for ix, _, _ in idx:
            ix.close()
