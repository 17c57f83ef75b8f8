"""Independent pure-Python restatement of skyvault's compaction path (small inputs only).

Written directly from the Rust sources, separately from oracle/skv_oracle.c, so that the two
restatements check each other (tests/test_oracle_vs_pyref.py). Test infrastructure only.

  decode   : runs::read_run_stream        src/runs.rs:517-628
  merge    : k_way::merge + HeapItem::cmp src/k_way.rs:14-33, :113-179
  filter   : Delete drop at Level::max    src/jobs/table_tree_compaction.rs:139-145
  encode   : runs::build_runs             src/runs.rs:166-282
  wal      : table split + prefix strip   src/jobs/wal_compaction.rs:66-174
  scan     : ScanFromRun over read_run_iter  src/cache_service.rs:97-151, src/runs.rs:400-510
"""
from __future__ import annotations

import heapq

EMPTY, VERSION, IO, FORMAT, INVALID_INPUT = 1, 2, 3, 4, 5
INTERNAL = 9
# mpsc::channel(100) of a WAL table task (wal_compaction.rs:113): once the task's build_runs has
# failed on an order error it drops its receiver; the job's sends to that table keep succeeding
# only while they can be buffered, and the 101st send after the failing op can never succeed.
# (Sends 1..100 may or may not fail -- a scheduling race; modelled here as succeeding.)
WAL_SENDS_AFTER_FAIL = 101


class Err(Exception):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code, self.msg = code, msg


def _utf8_ok(b: bytes) -> bool:
    try:
        b.decode("utf-8", "strict")
        return True
    except UnicodeDecodeError:
        return False


def decode(run: bytes, iterator: bool = False):
    """Generator of ('put'|'del', key, value) then raise Err (runs.rs:517-628). iterator=True:
    runs::read_run_iter's RunIterator (runs.rs:400-510), whose two length-EOF checks are Format
    errors with their own text instead of Io."""
    if len(run) == 0:
        raise Err(EMPTY, "Input list of operations cannot be empty")
    if run[0] != 1:
        raise Err(VERSION, f"Unsupported run version: {run[0]}")
    pos, n = 1, len(run)
    while pos < n:
        marker = run[pos]
        pos += 1
        if pos + 4 > n:
            if iterator:
                raise Err(FORMAT, "Data format error: Incomplete key length data")
            raise Err(IO, "I/O error: failed to fill whole buffer")
        klen = int.from_bytes(run[pos:pos + 4], "big")
        pos += 4
        if pos + klen > n:
            raise Err(FORMAT, "Data format error: Incomplete key data")
        key = run[pos:pos + klen]
        if not _utf8_ok(key):
            raise Err(FORMAT, "Data format error: Invalid UTF-8 in key")
        pos += klen
        if marker == 1:
            if pos + 4 > n:
                if iterator:
                    raise Err(FORMAT, "Data format error: Incomplete value length data")
                raise Err(IO, "I/O error: failed to fill whole buffer")
            vlen = int.from_bytes(run[pos:pos + 4], "big")
            pos += 4
            if pos + vlen > n:
                raise Err(FORMAT, "Data format error: Incomplete value data")
            yield ("put", key, run[pos:pos + vlen])
            pos += vlen
        elif marker == 2:
            yield ("del", key, None)
        else:
            raise Err(FORMAT, f"Data format error: Invalid marker byte: {marker}")


def stream_items(member_runs, iterator=False, gt=None):
    """flatten of the members' read_run_stream; Err surfaces as an ('err', Err) item. gt: keep only
    Ok items whose key is above it (ScanFromRun's try_filter, cache_service.rs:125-129)."""
    for r in member_runs:
        try:
            for it in decode(r, iterator):
                if gt is None or it[1] > gt:
                    yield it
        except Err as e:
            yield ("err", e, None)
            return


class _Key:
    """Heap entry: heapq is a min-heap, so order by (key asc, seq desc)."""

    __slots__ = ("item", "seq", "slot")

    def __init__(self, item, seq, slot):
        self.item, self.seq, self.slot = item, seq, slot

    def __lt__(self, o):
        if self.item[1] != o.item[1]:
            return self.item[1] < o.item[1]
        return self.seq > o.seq


def merge(streams, iterator=False, gt=None):
    """k_way::merge: yields emitted ops, raises Err at the first Err pulled."""
    its = [iter(stream_items(runs, iterator, gt)) for _, runs in streams]
    heap = []
    for i, (seq, _) in enumerate(streams):
        x = next(its[i], None)
        if x is None:
            continue
        if x[0] == "err":
            raise x[1]
        heapq.heappush(heap, _Key(x, seq, i))
    last = None
    while heap:
        top = heapq.heappop(heap)
        if last is None or top.item[1] != last:
            last = top.item[1]
            yield top.item
        x = next(its[top.slot], None)
        if x is None:
            continue
        if x[0] == "err":
            raise x[1]
        heapq.heappush(heap, _Key(x, top.seq, top.slot))


def build_runs(ops, max_size):
    """runs::build_runs -> list of (run_bytes, (min, max, size, puts, dels))."""
    out = []
    cur = bytearray()
    size = 0
    puts = dels = 0
    first = True
    last = None
    mn = mx = None
    for kind, k, v in ops:
        if last is not None and k <= last:
            raise Err(FORMAT, "Data format error: Operations must be sorted by key")
        last = k
        osz = 1 + 4 + len(k) + 4 + len(v) if kind == "put" else 1 + 4 + len(k)
        sw = size + 1 + osz if first else size + osz
        if not first and sw > max_size:
            out.append((bytes(cur), (mn, mx, size, puts, dels)))
            cur = bytearray()
            size = puts = dels = 0
            first = True
        if first:
            cur.append(1)
            size += 1
            mn = k
            first = False
        mx = k
        size += osz
        if kind == "put":
            cur += b"\x01" + len(k).to_bytes(4, "big") + k + len(v).to_bytes(4, "big") + v
            puts += 1
        else:
            cur += b"\x02" + len(k).to_bytes(4, "big") + k
            dels += 1
    if puts or dels:
        out.append((bytes(cur), (mn, mx, size, puts, dels)))
    return out


def _parse_i64(s: bytes):
    if not s:
        return None, "cannot parse integer from empty string"
    neg = False
    body = s
    if s[:1] in (b"+", b"-"):
        if len(s) == 1:
            return None, "invalid digit found in string"
        neg = s[:1] == b"-"
        body = s[1:]
    r = 0
    for c in body:
        if not (48 <= c <= 57):
            return None, "invalid digit found in string"
        r = r * 10 + (-(c - 48) if neg else (c - 48))
        if r > 2**63 - 1:
            return None, "number too large to fit in target type"
        if r < -(2**63):
            return None, "number too small to fit in target type"
    return r, None


def compact(streams, max_size, flags=0, races=None):
    """The job composition. Returns [(run_bytes, stats, table_id)], dropped_tables. races (a list):
    receives one entry per WAL table whose failed task races with 1..100 later sends to it."""
    seqs = [s for s, _ in streams]
    assert len(set(seqs)) == len(seqs)
    if flags & 2:
        return _wal(streams, max_size, races)
    ops = merge(streams)
    if flags & 1:
        ops = (o for o in ops if o[0] == "put")
    return [(b, st, 0) for b, st in build_runs(ops, max_size)], 0


def _wal(streams, max_size, races=None):
    result = []
    dropped = 0
    cur_table = None
    cur_ops = []
    fail_at = None  # index in cur_ops of the op whose order check fails the table's build_runs
    have = False

    def finish():
        nonlocal dropped
        if races is not None and fail_at is not None and 0 < len(cur_ops) - 1 - fail_at < WAL_SENDS_AFTER_FAIL:
            races.append(cur_table)
        try:
            runs = build_runs(cur_ops, max_size)
        except Err:
            dropped += 1
            return
        if len(runs) != 1:
            dropped += 1
            return
        result.append((runs[0][0], runs[0][1], cur_table))

    for kind, k, v in merge(streams):
        dot = k.find(b".")
        if dot < 0:
            raise Err(INVALID_INPUT, "Invalid input: Key does not follow 'table_id.key' format: " + k.decode())
        tid, perr = _parse_i64(k[:dot])
        if perr:
            raise Err(INVALID_INPUT, f"Invalid input: Invalid table ID '{k[:dot].decode()}': {perr}")
        strip = len(f"{tid}.")
        if not have or tid != cur_table:
            if have:
                finish()
            have = True
            cur_table = tid
            cur_ops = []
            fail_at = None
        cur_ops.append((kind, k[strip:], v))
        if fail_at is None and len(cur_ops) > 1 and cur_ops[-1][1] <= cur_ops[-2][1]:
            fail_at = len(cur_ops) - 1  # runs.rs:190-198 inside the table task
        if fail_at is not None and len(cur_ops) - 1 - fail_at == WAL_SENDS_AFTER_FAIL:
            raise Err(INTERNAL, "Internal error: Failed to send operation to table channel")  # :157-161
    if have:
        finish()
    return result, dropped


def scan(runs, start: bytes, max_results: int):
    """ScanFromRun (cache_service.rs:97-151): the response items [(kind, key, value)], or Err. Run i
    at SeqNo i64::MAX - i, read_run_iter, key > start, merged; the reader stops right after the
    max_results-th Put, so a merge error past that point is never seen."""
    if not 1 <= max_results <= 10000:
        raise Err(6, "max_results must be between 1 and 10000")
    items, puts = [], 0
    for op in merge([(2**63 - 1 - i, [r]) for i, r in enumerate(runs)], iterator=True, gt=start):
        items.append(op)
        puts += op[0] == "put"
        if puts >= max_results:
            break
    return items
