"""The pipelined host path (skv_compact with host inputs, skv_host.hip compact_host_pipelined):
key-range parts whose H2D, fused kernels and D2H overlap on three streams. Its outputs must be
the oracle's, byte for byte, whatever the cut keys (parts 2..17, equal keys across streams at the
cuts, empty parts), and a call the device poisons (a key decrease inside a part) or the host
rejects (a decrease across a cut) must end with the oracle's error through the serial path.

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

from test_gpu_parity import _diff, _run_both

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
    """variable record sizes: the host sees no fixed stride and never pipelines"""
    rng = random.Random(5)
    streams = []
    for s in range(4):
        keys = sorted(rng.sample(range(9000), 1500))
        streams.append((s + 1, [fmt.encode_run([fmt.put(f"k{i:06d}", b"v" * (1 + i % 7)) for i in keys])]))
    _check(dev, streams, 4 * MiB, 0, 4, expect_pipe=False)
    assert dev.timings()["host_parts"] == 0


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
    os.environ["SKV_TEST_FAIL_PART"] = str(fail_at)
    try:
        with pytest.raises(_abi.RunError) as ei:
            dev.compact(streams, 4 * MiB, 0)
    finally:
        os.environ.pop("SKV_TEST_FAIL_PART", None)
    assert ei.value.code == _abi.SKV_E_DEVICE and "injected failure" in ei.value.message
    for _ in range(3):  # the pool's buffer is taken and given back again on every call
        _check(dev, streams, 4 * MiB, 0, 6)
    _check(dev, _streams(rng, 3, 500, 4000), 4 * MiB, 0, 4)
