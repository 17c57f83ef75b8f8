"""The CPU restatement (oracle/skv_oracle.c) under AddressSanitizer + UndefinedBehaviorSanitizer
(host code only): oracle/sanitize_main.c drives skvo_compact over the oracle-vs-pyref case domain
(corrupt, truncated, unsorted, WAL, tombstones) with every run in an exact-size allocation, and
each outcome must equal the uninstrumented library's."""
import os
import struct
import subprocess

import pytest

from test_oracle_vs_pyref import _case

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE = os.path.join(os.path.dirname(HERE), "oracle")


def _fnv(h, b):
    for x in b:
        h = ((h ^ x) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _expect(oracle, streams, max_size, flags):
    import ctypes as C

    from skv._abi import SkvResult, StreamArgs

    sa = StreamArgs(streams)
    res = C.POINTER(SkvResult)()
    eb = C.create_string_buffer(512)
    rc = oracle.lib().skvo_compact(sa.ptr, sa.n, max_size, flags, C.byref(res), eb, 512)
    h = 0xCBF29CE484222325
    if rc == 0:
        r = res.contents
        h = _fnv(h, C.string_at(r.bytes, r.n_bytes) if r.n_bytes else b"")
        for i in range(r.n_runs):
            h = _fnv(h, C.string_at(C.addressof(r.runs[i]), 80))
        oracle.lib().skvo_result_free(res)
    else:
        h = _fnv(h, eb.value)
    return f"rc {rc} {h:016x}"


def test_oracle_under_asan_ubsan(oracle, tmp_path):
    try:
        subprocess.check_call(["make", "-s", "-C", ORACLE, "skv_oracle_asan"])
    except (OSError, subprocess.CalledProcessError) as e:
        pytest.skip(f"sanitizer build unavailable: {e}")
    cases = [_case(seed) for seed in range(300)]
    blob = bytearray()
    for streams, max_size, flags in cases:
        blob += struct.pack("<IQI", len(streams), max_size, flags)
        for seq, runs in streams:
            blob += struct.pack("<qI", seq, len(runs))
            for r in runs:
                blob += struct.pack("<Q", len(r)) + bytes(r)
    path = tmp_path / "cases.bin"
    path.write_bytes(bytes(blob))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    out = subprocess.run([os.path.join(ORACLE, "skv_oracle_asan"), str(path)], capture_output=True, text=True,
                         env=env, timeout=600)
    assert out.returncode == 0, out.stderr[-4000:]
    got = out.stdout.splitlines()
    assert len(got) == len(cases)
    exp = [_expect(oracle, *c) for c in cases]
    assert got == exp
