"""GPU parity at BASELINE.json's full sizes, through the device-resident entry point that
bench.py measures (skv_compact_dev), against the oracle (oracle/skv_oracle.c).

  config 2A / 2B  64 x 1 run x 238,821 records (4.0 GiB), built in HBM exactly as bench.py
                  builds them: R = 15.3 M records, above the fused path's 2^22-record sampling
                  switch. The oracle compacts the whole input in one call; every output byte and
                  every one of the ~1,025 descriptors must match.
  config 5        10^6 WAL runs x 83 records (3.8 GiB), SKV_SPLIT_BY_TABLE, at max 2^62 (one run
                  per table) and at the jobs' 4 MiB (the exactly-one-run rule drops every table).
                  The oracle runs per group of tables (whole tables are independent in
                  wal_compaction.rs:66-174: the merged order visits them one after another), the
                  groups in parallel threads; concatenated in table order they are the full
                  expected output.
  config 3F       256 x 1 run x 256 MiB (64 GiB, 206 M records, variable keys, 10 % Deletes),
                  flags 0 and SKV_DROP_TOMBSTONES. The oracle merges 256 disjoint key ranges
                  separately (k_way::merge restricted to a key range is the merge of the streams'
                  sub-ranges; the Delete filter is per op) with an unbounded max run size, and
                  ONE streaming build_runs (pyoracle.StreamBuilder, runs.rs:166-282) splits their
                  concatenation into 4 MiB runs — so the greedy split, the order check and
                  StatsV1 carry across ranges exactly as in one call. Every output byte and
                  descriptor is compared.

Device output is read back in slices with hipMemcpy, so host memory stays a few GiB (config 2:
~20 GiB for the one-call oracle).
"""
import ctypes as C
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from skv import _abi
from skv.api import Compactor

import pyoracle

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
MiB = 1 << 20
MAX_RUN = 4 * MiB
SEED = 0x5EEDC0DE  # bench.rank_seed(0): the bench's own rank-0 input
THREADS = int(os.environ.get("SKV_TEST_THREADS", "12"))


@pytest.fixture(scope="module")
def torch():
    t = pytest.importorskip("torch")
    t.cuda.init()
    return t


@pytest.fixture(scope="module")
def dev(torch):
    c = Compactor(0, profiling=True)
    yield c
    c.close()


_hip = None
_PROGRESS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "fullsize_progress.log")


def _progress(msg: str):
    """A line per step to gpurun_out/ (pytest captures stdout/stderr; a GPU-box run that writes
    nothing for minutes is taken to be hung)."""
    import time

    os.makedirs(os.path.dirname(_PROGRESS), exist_ok=True)
    with open(_PROGRESS, "a") as f:
        f.write(f"{time.strftime('%H:%M:%S')} {msg}\n")


def d2h(ptr: int, n: int) -> np.ndarray:
    """n bytes at device address ptr -> a host numpy array (hipMemcpy, device-to-host)."""
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")
    out = np.empty(n, dtype=np.uint8)
    if n:
        rc = _hip.hipMemcpy(C.c_void_p(out.ctypes.data), C.c_void_p(ptr), C.c_size_t(n), 2)
        assert rc == 0, f"hipMemcpy D2H failed: {rc}"
    return out


def _first_diff(a: np.ndarray, b: np.ndarray):
    n = min(a.size, b.size)
    d = np.nonzero(a[:n] != b[:n])[0]
    return int(d[0]) if d.size else n


def _compare_bytes(res, pos: int, exp: np.ndarray, what: str, chunk: int = 1 << 30):
    for q in range(0, exp.size, chunk):
        part = exp[q:q + chunk]
        got = d2h(res.dev_ptr + pos + q, part.size)
        if not np.array_equal(got, part):
            raise AssertionError(f"{what}: output byte {pos + q + _first_diff(got, part)} differs")


# ------------------------------------------------------------------------------------------
# config 2A / 2B: one oracle call over the whole 4 GiB input


@pytest.mark.parametrize("variant", ["A", "B"])
def test_config2_full_size(dev, torch, variant):
    from skv.devgen import make_cfg2_on_device

    device = torch.device("cuda", 0)
    _progress(f"config 2{variant}: generating")
    runs = make_cfg2_on_device(device, SEED, 64, 238821, 256, variant)
    streams = [(s + 1, [(r.data_ptr(), r.numel())]) for s, r in enumerate(runs)]
    res = dev.compact_dev(streams, MAX_RUN, 0)
    t = dev.timings()
    assert t["path"] == _abi.PATH_FUSED, t
    assert res.in_records == 64 * 238821 and res.in_records >= 1 << 22  # the fused level-1 switch
    host = [r.cpu().numpy() for r in runs]
    del runs
    sa = _abi.stream_table(np.arange(1, 65), [h.ctypes.data for h in host], [h.size for h in host])
    _progress(f"config 2{variant}: oracle")
    exp, descs, info = pyoracle.compact_np(sa, MAX_RUN, 0)
    _progress(f"config 2{variant}: compare")
    assert (res.n_bytes, res.n_runs, res.out_records) == (exp.size, len(descs), info["out_records"])
    _compare_bytes(res, 0, exp, f"config 2{variant}")
    assert res.descs == descs
    if variant == "A":
        assert res.n_runs == 1025 and res.out_records == res.in_records
    res.free()


# ------------------------------------------------------------------------------------------
# config 4: eight independent config-2A compactions at once (orchestrator_service.rs:119-170
# schedules per-table / per-level jobs independently), one ctx + worker thread each


def test_config4_eight_compactions_at_once(torch):
    """BASELINE config 4's workload on the visible devices: 8 config-2A compactions (64 x 238,821
    records, 4 GiB each, the bench's rank seeds 0..7) submitted together to skv.multi.MultiCompactor
    with one ctx and one worker thread per job (on a one-GPU box all eight share device 0: 32 GiB of
    inputs and 8 output buffers in HBM, eight calls in flight on eight HIP streams). Every job's
    bytes and descriptors are compared with its own oracle call."""
    from skv.devgen import make_cfg2_on_device
    from skv.multi import MultiCompactor

    n_dev = torch.cuda.device_count()
    seeds = [SEED + 1000 * j for j in range(8)]  # bench.rank_seed(0..7)
    inputs = []
    for j, sd in enumerate(seeds):
        _progress(f"config 4: generating job {j}")
        inputs.append(make_cfg2_on_device(torch.device("cuda", j % n_dev), sd, 64, 238821, 256, "A"))

    def keep(comp, res):  # on the worker thread, before any later call on that ctx
        return res, comp.timings()

    _progress("config 4: 8 jobs submitted")
    with MultiCompactor([j % n_dev for j in range(8)]) as mc:
        futs = [mc.submit([(s + 1, [(r.data_ptr(), r.numel())]) for s, r in enumerate(runs)], MAX_RUN, 0,
                          entry="compact_dev", then=keep) for runs in inputs]
        results = [f.result() for f in futs]
        try:
            assert len({w.ident for w in mc._workers}) == 8
            _progress("config 4: compare")

            def oracle(j):  # the C oracle releases the GIL: two jobs' oracles at a time
                host = [r.cpu().numpy() for r in inputs[j]]
                sa = _abi.stream_table(np.arange(1, 65), [h.ctypes.data for h in host], [h.size for h in host])
                return pyoracle.compact_np(sa, MAX_RUN, 0)

            with ThreadPoolExecutor(2) as ex:
                pending = {j: ex.submit(oracle, j) for j in range(2)}
                for j, (res, t) in enumerate(results):
                    exp, descs, info = pending.pop(j).result()
                    if j + 2 < 8:
                        pending[j + 2] = ex.submit(oracle, j + 2)
                    assert t["path"] == _abi.PATH_FUSED, (j, t)
                    assert (res.n_bytes, res.n_runs, res.out_records) == (exp.size, len(descs), info["out_records"]), j
                    _compare_bytes(res, 0, exp, f"config 4 job {j}")
                    assert res.descs == descs, j
                    del exp
                    res.free()
                    _progress(f"config 4: job {j} bit-exact")
        finally:
            for res, _ in results:  # before the workers destroy their ctxs
                res.free()


# ------------------------------------------------------------------------------------------
# the host-memory entry point (skv_compact) at BASELINE size, default pipeline thresholds


@pytest.fixture
def default_pipe_env():
    """skv_compact with its shipped thresholds: no SKV_HOST_PIPE* / SKV_HOST_PARTS override."""
    keys = ("SKV_HOST_PIPE", "SKV_HOST_PIPE_MIN", "SKV_HOST_PARTS")  # (test hooks are cleared per test)
    old = {k: os.environ.pop(k, None) for k in keys}
    yield
    for k, v in old.items():
        if v is not None:
            os.environ[k] = v


def _pinned_copies(torch, runs):
    return [r.cpu().pin_memory() for r in runs]


def _check_host_result(hr, exp, descs, info, what):
    assert (hr.n_bytes, hr.n_runs, hr.out_records) == (exp.size, len(descs), info["out_records"]), what
    for q in range(0, exp.size, 1 << 30):
        got = hr.host_bytes(q, min(1 << 30, exp.size - q))
        part = exp[q:q + got.size]
        if not np.array_equal(got, part):
            raise AssertionError(f"{what}: output byte {q + _first_diff(got, part)} differs")
    assert hr.descs == descs, what


def test_config2_host_entry_full_size(dev, torch, default_pipe_env):
    """config 2A through skv_compact with pinned host inputs (storage.rs:226-250 get_run -> compact
    -> put_run, table_buffer_compaction.rs:103-121): 4 GiB, so the fused key-range pipeline runs
    with its own part count (15 parts); every byte and descriptor equal to the oracle's."""
    from skv.devgen import make_cfg2_on_device

    device = torch.device("cuda", 0)
    _progress("config 2A host entry: generating")
    runs = make_cfg2_on_device(device, SEED, 64, 238821, 256, "A")
    host = _pinned_copies(torch, runs)
    del runs
    torch.cuda.empty_cache()
    streams = [(s + 1, [(h.data_ptr(), h.numel())]) for s, h in enumerate(host)]
    hr = dev.compact_host(streams, MAX_RUN, 0)
    t = dev.timings()
    assert t["host_parts"] >= 2, t  # the pipeline, not the serial copies
    _progress(f"config 2A host entry: {t['host_parts']} parts; oracle")
    arrs = [h.numpy() for h in host]
    sa = _abi.stream_table(np.arange(1, 65), [a.ctypes.data for a in arrs], [a.size for a in arrs])
    exp, descs, info = pyoracle.compact_np(sa, MAX_RUN, 0)
    _check_host_result(hr, exp, descs, info, "config 2A host entry")
    assert hr.n_runs == 1025
    hr.free()


def test_config2_split_full_size(torch, default_pipe_env):
    """config 2B (~37 % superseded) through skv_compact_split over 4 ctxs (one
    compaction as 4 key-range shards, 4 parts each, counts exchanged, survivors placed by the
    global split): every byte and descriptor equal to the oracle's."""
    from skv.api import compact_split
    from skv.devgen import make_cfg2_on_device

    device = torch.device("cuda", 0)
    _progress("config 2B split: generating")
    runs = make_cfg2_on_device(device, SEED, 64, 238821, 256, "B")
    host = _pinned_copies(torch, runs)
    del runs
    torch.cuda.empty_cache()
    streams = [(s + 1, [(h.data_ptr(), h.numel())]) for s, h in enumerate(host)]
    cs = [Compactor(0) for _ in range(4)]
    try:
        hr = compact_split(cs, streams, MAX_RUN, 0, keep=True)
        t = cs[0].timings()
        assert t["host_parts"] >= 8 and t["host_parts"] % 4 == 0, t  # 4 shards of parts, not skv_compact
        _progress("config 2B split: oracle")
        arrs = [h.numpy() for h in host]
        sa = _abi.stream_table(np.arange(1, 65), [a.ctypes.data for a in arrs], [a.size for a in arrs])
        exp, descs, info = pyoracle.compact_np(sa, MAX_RUN, 0)
        _check_host_result(hr, exp, descs, info, "config 2B split")
        hr.free()
    finally:
        for c in cs:
            c.close()


def test_config3_host_entry_full_size(dev, torch, default_pipe_env):
    """config 3's shape (256 streams, variable 8-128 B keys, 10 % Deletes) at 256 x 16 MiB (3.7 GiB)
    through skv_compact with pinned host inputs: the general key-range pipeline with its own part
    count (~1 GiB parts) and the open output run carried across parts. Flags 0 and the Delete
    filter; every byte and descriptor equal to the oracle's."""
    from skv.devgen import make_cfg3_on_device

    device = torch.device("cuda", 0)
    _progress("config 3 host entry: generating")
    runs = make_cfg3_on_device(device, SEED, 256, 16)
    host = _pinned_copies(torch, runs)
    del runs
    torch.cuda.empty_cache()
    streams = [(s + 1, [(h.data_ptr(), h.numel())]) for s, h in enumerate(host)]
    arrs = [h.numpy() for h in host]
    sa = _abi.stream_table(np.arange(1, 257), [a.ctypes.data for a in arrs], [a.size for a in arrs])
    for flags in (0, _abi.SKV_DROP_TOMBSTONES):
        hr = dev.compact_host(streams, MAX_RUN, flags)
        t = dev.timings()
        assert t["host_parts"] >= 2 and t["path"] == _abi.PATH_GENERAL, t
        _progress(f"config 3 host entry flags {flags}: {t['host_parts']} parts; oracle")
        exp, descs, info = pyoracle.compact_np(sa, MAX_RUN, flags)
        _check_host_result(hr, exp, descs, info, f"config 3 host entry flags {flags}")
        hr.free()


def test_config3_split_full_size(torch, default_pipe_env):
    """config 3's shape at 256 x 16 MiB (3.7 GiB) through skv_compact_split over 4 ctxs with 3 parts
    each (SURVEY §8(e) for variable-length records: parallel merges, build_runs' split carried from
    part to part). Flags 0 and the Delete filter; every byte and descriptor equal to the oracle's."""
    from skv.api import compact_split
    from skv.devgen import make_cfg3_on_device

    device = torch.device("cuda", 0)
    _progress("config 3 split: generating")
    runs = make_cfg3_on_device(device, SEED + 7, 256, 16)
    host = _pinned_copies(torch, runs)
    del runs
    torch.cuda.empty_cache()
    streams = [(s + 1, [(h.data_ptr(), h.numel())]) for s, h in enumerate(host)]
    arrs = [h.numpy() for h in host]
    sa = _abi.stream_table(np.arange(1, 257), [a.ctypes.data for a in arrs], [a.size for a in arrs])
    cs = [Compactor(0) for _ in range(4)]
    os.environ["SKV_SPLIT_PARTS"] = "3"
    try:
        for flags in (0, _abi.SKV_DROP_TOMBSTONES):
            hr = compact_split(cs, streams, MAX_RUN, flags, keep=True)
            t = cs[0].timings()
            assert t["host_parts"] >= 8 and t["path"] == _abi.PATH_GENERAL, t
            _progress(f"config 3 split flags {flags}: {t['host_parts']} parts; oracle")
            exp, descs, info = pyoracle.compact_np(sa, MAX_RUN, flags)
            _check_host_result(hr, exp, descs, info, f"config 3 split flags {flags}")
            hr.free()
    finally:
        os.environ.pop("SKV_SPLIT_PARTS", None)
        for c in cs:
            c.close()


# ------------------------------------------------------------------------------------------
# config 5: 10^6 WAL runs, oracle per group of whole tables


def _table_rank(n_tables: int = 64) -> np.ndarray:
    """rank of table t in merged (bytewise key) order: "{t}." sorts like str(t)."""
    order = sorted(range(n_tables), key=str)
    rank = np.empty(n_tables, dtype=np.int64)
    rank[order] = np.arange(n_tables)
    return rank


def _wal_group_inputs(host: np.ndarray, groups: int):
    """Per group of consecutive tables (in key order): one host buffer holding, for every WAL run
    with records of those tables, a version byte + those records, and its stream table."""
    n, rl = host.shape
    recs = host[:, 1:].reshape(n, (rl - 1) // 49, 49)
    k0, k1 = recs[:, :, 5].astype(np.int64) - 48, recs[:, :, 6]
    table = np.where(k1 == ord("."), k0, 10 * k0 + (k1.astype(np.int64) - 48))
    grp = _table_rank()[table] // (64 // groups)
    assert (np.diff(grp, axis=1) >= 0).all()  # each run visits the tables in key order
    for g in range(groups):
        mask = grp == g
        cnt = mask.sum(axis=1)
        live = np.nonzero(cnt)[0]
        c = cnt[live]
        flat = recs[mask].reshape(-1)
        starts = np.zeros(live.size, dtype=np.int64)
        starts[1:] = np.cumsum(49 * c[:-1])
        buf = np.insert(flat, starts, 1).astype(np.uint8)
        run_off = starts + np.arange(live.size)
        yield buf, live + 1, buf.ctypes.data + run_off.astype(np.uint64), 1 + 49 * c


def _wal_oracle(host: np.ndarray, max_run: int, groups: int = 16):
    def one(args):
        buf, seqs, ptrs, lens = args
        sa = _abi.stream_table(seqs, ptrs, lens)
        data, descs, info = pyoracle.compact_np(sa, max_run, _abi.SKV_SPLIT_BY_TABLE)
        _progress(f"config 5: table group of {len(seqs)} runs done")
        del buf
        return data, descs, info

    with ThreadPoolExecutor(THREADS) as ex:
        parts = list(ex.map(one, _wal_group_inputs(host, groups)))
    data = np.concatenate([p[0] for p in parts]) if parts else np.empty(0, np.uint8)
    descs, base = [], 0
    for d, ds, _ in parts:
        for x in ds:
            descs.append((x[0] + base, x[1], x[2], x[3], x[4] + base, x[5], x[6] + base, x[7], x[8]))
        base += d.size
    dropped = sum(p[2]["dropped_tables"] for p in parts)
    out_records = sum(p[2]["out_records"] for p in parts)
    return data, descs, dropped, out_records


def test_config5_full_size(dev, torch):
    from skv.devgen import make_cfg5_on_device

    n_streams = 1_000_000
    device = torch.device("cuda", 0)
    _progress("config 5: generating")
    buf = make_cfg5_on_device(device, SEED, n_streams)
    rl = buf.shape[1]
    sa = _abi.stream_table(np.arange(1, n_streams + 1), buf.data_ptr() + rl * np.arange(n_streams, dtype=np.uint64),
                           np.full(n_streams, rl))
    host = buf.cpu().numpy()
    for max_run in (1 << 62, MAX_RUN):
        res = dev.compact_dev(sa, max_run, _abi.SKV_SPLIT_BY_TABLE)
        assert dev.timings()["sorted"] == 1  # 10^6-way fan-in takes the record sort
        raw = res._res.contents
        exp, descs, dropped, out_records = _wal_oracle(host, max_run)
        assert (res.n_bytes, res.n_runs, raw.dropped_tables, res.out_records) == \
            (exp.size, len(descs), dropped, out_records)
        _compare_bytes(res, 0, exp, f"config 5 max {max_run}")
        assert res.descs == descs
        if max_run == MAX_RUN:  # ~63 MB per table > 4 MiB: the one-run rule drops all of them
            assert res.n_runs == 0 and dropped == 64
        else:
            assert res.n_runs == 64 and dropped == 0
        res.free()


# ------------------------------------------------------------------------------------------
# config 3 at 256 x 256 MiB: key-range merges + one streaming build_runs


@pytest.fixture(scope="module")
def cfg3_full(torch):
    from skv.devgen import make_cfg3_full_on_device

    device = torch.device("cuda", 0)
    n_streams, run_mib = 256, 256
    _progress("config 3F: generating")
    runs, index = make_cfg3_full_on_device(device, SEED, n_streams, run_mib, with_index=True)
    _progress("config 3F: generated")
    n = (run_mib << 20) // 333
    universe = n * n_streams * 2
    P = 256  # key ranges (id ranges: keys sort like their ids)
    bounds = torch.linspace(0, universe, P + 1, device=device).to(torch.int64)
    bounds[-1] = universe
    cuts = []
    for r, (ids, off) in zip(runs, index):
        pos = torch.searchsorted(ids, bounds)
        off_ext = torch.cat([off, torch.tensor([r.numel()], device=device, dtype=off.dtype)])
        cuts.append(off_ext[pos].cpu().numpy())
    del index
    torch.cuda.synchronize()
    yield runs, np.stack(cuts), P
    del runs


def _range_input(torch, runs, cuts, p):
    """Key range p of every stream as one host buffer (version byte + the range's records per
    non-empty stream) and its stream table."""
    one = torch.ones(1, dtype=torch.uint8, device=runs[0].device)
    parts, seqs, lens = [], [], []
    for s, r in enumerate(runs):
        a, b = int(cuts[s, p]), int(cuts[s, p + 1])
        if b > a:
            parts += [one, r[a:b]]
            seqs.append(s + 1)
            lens.append(1 + b - a)
    if not parts:
        return None
    buf = torch.cat(parts).cpu().numpy()
    offs = np.zeros(len(lens), dtype=np.uint64)
    offs[1:] = np.cumsum(lens[:-1])
    return buf, np.array(seqs), buf.ctypes.data + offs, np.array(lens)


@pytest.mark.parametrize("flags", [0, _abi.SKV_DROP_TOMBSTONES], ids=["flags0", "drop_tombstones"])
def test_config3_full_size(dev, torch, cfg3_full, flags):
    runs, cuts, P = cfg3_full
    streams = [(s + 1, [(r.data_ptr(), r.numel())]) for s, r in enumerate(runs)]
    res = dev.compact_dev(streams, MAX_RUN, flags)
    assert dev.timings()["path"] == _abi.PATH_GENERAL
    in_bytes = sum(r.numel() for r in runs)
    assert res.in_bytes == in_bytes and in_bytes > 63e9  # 256 x ~249 MB

    def merge_range(p):
        inp = _range_input(torch, runs, cuts, p)
        if inp is None:
            return None
        buf, seqs, ptrs, lens = inp
        data, _, _ = pyoracle.compact_np(_abi.stream_table(seqs, ptrs, lens), 1 << 62, flags)
        return data

    sb = pyoracle.StreamBuilder(MAX_RUN)
    pos = 0
    window = 2 * THREADS  # key ranges in flight (each ~250 MB in + out)
    with ThreadPoolExecutor(THREADS) as ex:
        futs = {p: ex.submit(merge_range, p) for p in range(min(window, P))}
        for p in range(P):
            data = futs.pop(p).result()
            if p + window < P:
                futs[p + window] = ex.submit(merge_range, p + window)
            if data is None or data.size == 0:
                continue
            out = sb.feed(data)
            _compare_bytes(res, pos, out, f"config 3F range {p}")
            if p % 16 == 0:
                _progress(f"config 3F flags {flags}: range {p}/{P} ok")
            pos += out.size
    tail, descs = sb.finish()
    tail = np.frombuffer(tail, dtype=np.uint8)
    _compare_bytes(res, pos, tail, "config 3F tail")
    assert res.n_bytes == pos + tail.size
    assert res.descs == descs
    assert all(d[1] <= MAX_RUN for d in descs)
    if flags:
        assert all(d[3] == 0 for d in descs)
    res.free()


def test_config5_host_entry_full_size(dev, torch):
    """config 5 through skv_compact with the 10^6 WAL runs in pinned host memory (storage.rs:183-250
    get_run -> compact -> put_run, wal_compaction.rs:18-51): past 2^16 runs the call takes the serial
    path (the many-run pipeline measured slower and was removed in round 6); bytes
    and descriptors equal to the per-table-group oracle at both max sizes."""
    from skv.devgen import make_cfg5_on_device

    n_streams = 1_000_000
    buf = make_cfg5_on_device(torch.device("cuda", 0), SEED + 5, n_streams)
    host_t = buf.cpu().pin_memory()
    del buf
    rl = host_t.shape[1]
    sa = _abi.stream_table(np.arange(1, n_streams + 1), host_t.data_ptr() + rl * np.arange(n_streams, dtype=np.uint64),
                           np.full(n_streams, rl))
    host = host_t.numpy()
    _config5_host(dev, sa, host)


def _config5_host(dev, sa, host):
    for max_run in (1 << 62, MAX_RUN):
        _progress(f"config 5 host entry max {max_run}: device")
        hr = dev.compact_host(sa, max_run, _abi.SKV_SPLIT_BY_TABLE)
        t = dev.timings()
        assert t["host_parts"] == 0, t  # past 2^16 runs: the serial path
        _progress(f"config 5 host entry: {t['host_parts']} parts; oracle")
        exp, descs, dropped, out_records = _wal_oracle(host, max_run)
        raw = hr._res.contents
        assert (hr.n_bytes, hr.n_runs, raw.dropped_tables, hr.out_records) == (exp.size, len(descs), dropped, out_records)
        if exp.size:
            got = hr.host_bytes(0, exp.size)
            assert np.array_equal(got, exp), f"config 5 host entry: byte {_first_diff(got, exp)} differs"
        assert hr.descs == descs
        hr.free()
