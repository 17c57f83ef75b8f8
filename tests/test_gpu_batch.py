"""GPU parity of the writer-side batch encode (skv_encode_batch, include/skv.h): the batch's ops
in request order -> BTreeMap by key (the last op of a key wins) -> build_runs
(writer_service.rs:148-162), bit-exact against the CPU restatement (oracle/pyoracle.encode_batch).
The device path is the record sort (skv_sort.hip) with the tie order reversed."""
import random

import pytest

from skv import _abi, gen
from skv import format as fmt
from skv.api import Compactor

import pyoracle

pytestmark = pytest.mark.gpu
MiB = 1 << 20


@pytest.fixture(scope="module")
def dev():
    torch = pytest.importorskip("torch")
    torch.cuda.init()
    c = Compactor(0, profiling=True)
    yield c
    c.close()


def _norm(runs):
    return [(r.data, r.stats.min_key, r.stats.max_key, r.stats.put_count, r.stats.delete_count) for r in runs]


def _both(dev, run, max_size):
    try:
        exp = ("ok", _norm(pyoracle.encode_batch(run, max_size)))
    except _abi.RunError as e:
        exp = ("err", e.code, e.message)
    try:
        got = ("ok", _norm(dev.encode_batch(run, max_size)))
    except _abi.RunError as e:
        got = ("err", e.code, e.message)
    return exp, got


def _batch(r: random.Random, n: int, universe: int, klen=(1, 40), vlen=(0, 30), deletes=0.2):
    ops = []
    for _ in range(n):
        k = f"k{r.randrange(universe):07d}" + "x" * r.randint(0, klen[1] - 8)
        if r.random() < deletes:
            ops.append(fmt.delete(k))
        else:
            ops.append(fmt.put(k, bytes(r.getrandbits(8) for _ in range(r.randint(*vlen)))))
    return fmt.encode_run(ops)


@pytest.mark.parametrize("n,universe,max_size", [
    (1, 10, 4 * MiB), (10, 3, 4 * MiB), (500, 100, 4 * MiB), (5000, 1000, 1 << 14), (20000, 50000, 4 * MiB),
    (3000, 10, 200), (4096, 4096, 1 << 16), (4097, 1, 4 * MiB),
])
def test_batch_matches_oracle(dev, n, universe, max_size):
    r = random.Random(n * 7 + universe)
    exp, got = _both(dev, _batch(r, n, universe), max_size)
    assert exp == got


def test_batch_fixed_shape_and_long_shared_keys(dev):
    r = random.Random(3)
    # fixed-stride ops (the fast parse path): 24 B keys, 8 B values, many repeats
    ops = [fmt.put(f"t{r.randrange(900):05d}-" + "p" * 17, r.randbytes(8)) for _ in range(30000)]
    exp, got = _both(dev, fmt.encode_run(ops), 4 * MiB)
    assert exp == got
    # keys sharing 40 bytes, prefixes of each other
    base = "tenant/ns/partition-000/shard-0000001/x/"
    ops = [fmt.put(base + "".join(r.choice("ab") for _ in range(r.randint(0, 20))), b"v") for _ in range(8000)]
    exp, got = _both(dev, fmt.encode_run(ops), 1 << 15)
    assert exp == got


def test_batch_errors(dev):
    good = fmt.encode_run([fmt.put("b", b"1"), fmt.put("a", b"2")])
    for bad in (b"", b"\x02" + good[1:], good[:-1], good[:4], good + b"\x07"):
        exp, got = _both(dev, bad, 4 * MiB)
        assert exp == got, (bad, exp, got)


def test_batch_reference_semantics(dev):
    """BTreeMap replacement: a later Put or Delete replaces an earlier op of the same key."""
    ops = [fmt.put("k", b"old"), fmt.put("a", b"1"), fmt.delete("k"), fmt.put("z", b"9"), fmt.put("k", b"new"),
           fmt.delete("z")]
    runs = dev.encode_batch(fmt.encode_run(ops), 4 * MiB)
    assert len(runs) == 1
    assert runs[0].data == fmt.encode_run([fmt.put("a", b"1"), fmt.put("k", b"new"), fmt.delete("z")])
