"""Writes the golden fixtures under tests/golden/.

kat.json — known-answer tests transcribed from the reference's own unit tests (expected
values are the ones those tests assert; citations are /root/reference paths):
  runs.rs:775-802   test_create_run_simple            (the 39-byte golden run)
  runs.rs:805-813   test_create_run_with_duplicates   (Format error)
  runs.rs:816-820   test_create_run_empty_input       (no runs)
  runs.rs:823-883   test_search_run_{found,tombstone,not_found} (one run; search results)
  runs.rs:886-911   test_create_run_with_iterator     (identical bytes)
  runs.rs:914-1000  test_create_multiple_runs_due_to_size (52 runs of 1,048,577 B at max 2 MiB)
  k_way.rs:42-107   test_heap_item_ordering_*         (pop order a(2), a(1), b, c)
  k_way.rs:186-226  test_merge                        (a:[10], b:[20], c:[3])
  cache_service.rs:349-391 test_scan_from_run_multiple_runs (apple@run1, banana@run2, Delete cherry)
plus decode-error vectors hand-derived from runs.rs:537-624 (each RunError the decoder can
yield, in its check order).

compact_cases.json — generated compaction cases: inputs and outputs produced by the C
restatement (oracle/) and required to agree with the independent Python restatement
(tests/pyref.py) before they are written. Run from the repo root:
    python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "skyvault-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import pyref  # noqa: E402
from skv import format as fmt  # noqa: E402
from skv import gen  # noqa: E402

KiB, MiB = 1 << 10, 1 << 20


def h(b: bytes) -> str:
    return bytes(b).hex()


def op_json(op):
    is_put, k, v = op
    return {"put": bool(is_put), "key": h(k), "val": h(v) if is_put else None}


def kats():
    P, D = fmt.put, fmt.delete
    k = []
    k.append({
        "name": "test_create_run_simple", "ref": "src/runs.rs:775-802", "kind": "build_runs",
        "max": 1024, "ops": [op_json(P("apple", b"red")), op_json(P("banana", b"yellow"))],
        "expect": {"runs": [{"hex": "01" "01" "00000005" "6170706c65" "00000003" "726564"
                                    "01" "00000006" "62616e616e61" "00000006" "79656c6c6f77",
                             "min_key": "apple", "max_key": "banana", "size_bytes": 39,
                             "put_count": 2, "delete_count": 0}]},
    })
    k.append({
        "name": "test_create_run_with_duplicates", "ref": "src/runs.rs:805-813", "kind": "build_runs",
        "max": 1024, "ops": [op_json(P("apple", b"green")), op_json(P("apple", b"red"))],
        "expect": {"error": "Format", "message": "Data format error: Operations must be sorted by key"},
    })
    k.append({
        "name": "test_create_run_empty_input", "ref": "src/runs.rs:816-820", "kind": "build_runs",
        "max": 1024, "ops": [], "expect": {"runs": []},
    })
    k.append({
        "name": "test_search_run_found", "ref": "src/runs.rs:823-836", "kind": "build_runs",
        "max": 1024,
        "ops": [op_json(P("apple", b"red")), op_json(P("banana", b"yellow")), op_json(P("cherry", b"red"))],
        "expect": {"n_runs": 1, "search": {"banana": ["found", h(b"yellow")], "apple": ["found", h(b"red")],
                                           "cherry": ["found", h(b"red")]}},
    })
    k.append({
        "name": "test_search_run_tombstone", "ref": "src/runs.rs:838-851", "kind": "build_runs",
        "max": 1024,
        "ops": [op_json(P("apple", b"red")), op_json(D("banana")), op_json(P("cherry", b"red"))],
        "expect": {"n_runs": 1, "search": {"banana": ["tombstone", None], "apple": ["found", h(b"red")]}},
    })
    k.append({
        "name": "test_search_run_not_found", "ref": "src/runs.rs:853-869", "kind": "build_runs",
        "max": 1024, "ops": [op_json(P("banana", b"yellow")), op_json(P("date", b"brown"))],
        "expect": {"n_runs": 1, "search": {"apple": ["not_found", None], "cherry": ["not_found", None],
                                           "elderberry": ["not_found", None]}},
    })
    k.append({
        "name": "test_create_run_with_iterator", "ref": "src/runs.rs:886-911", "kind": "build_runs",
        "max": 1024, "ops": [op_json(P("apple", b"red")), op_json(P("banana", b"yellow"))],
        "expect": {"same_as": "test_create_run_simple"},
    })
    # 52 ops whose record size is exactly 1 MiB (value 1,048,553 zero bytes, key "key_%010d"),
    # at max 2 MiB: 1 + 2*2^20 > 2^21, so every run holds one record (runs.rs:211-219).
    k.append({
        "name": "test_create_multiple_runs_due_to_size", "ref": "src/runs.rs:914-1000",
        "kind": "build_runs_generated", "max": 2 * MiB,
        "gen": {"count": 52, "key_fmt": "key_%010d", "record_size": MiB},
        "expect": {"n_runs": 52, "size_bytes_each": MiB + 1},
    })
    k.append({
        "name": "test_heap_item_ordering_binary_heap", "ref": "src/k_way.rs:71-107", "kind": "merge",
        # each heap entry as its own single-op stream; the merge emits in pop order with dedup
        "streams": [[1, [op_json(P("c", b"\x01"))]], [11, [op_json(P("a", b"\x01"))]],
                    [21, [op_json(P("b", b"\x01"))]], [22, [op_json(P("a", b"\x02"))]]],
        "expect": {"ops": [op_json(P("a", b"\x02")), op_json(P("b", b"\x01")), op_json(P("c", b"\x01"))]},
    })
    k.append({
        "name": "test_merge", "ref": "src/k_way.rs:186-226", "kind": "merge",
        "streams": [[1, [op_json(P("a", b"\x01")), op_json(P("c", b"\x03"))]],
                    [2, [op_json(P("a", b"\x0a")), op_json(P("b", b"\x14"))]]],
        "expect": {"ops": [op_json(P("a", b"\x0a")), op_json(P("b", b"\x14")), op_json(P("c", b"\x03"))]},
    })
    i64max = 2**63 - 1
    k.append({
        "name": "test_scan_from_run_multiple_runs", "ref": "src/cache_service.rs:349-391", "kind": "merge",
        "streams": [[i64max, [op_json(P("banana", b"green_from_run2")), op_json(D("cherry"))]],
                    [i64max - 1, [op_json(P("apple", b"red_from_run1")), op_json(P("banana", b"yellow_from_run1"))]]],
        "expect": {"ops": [op_json(P("apple", b"red_from_run1")), op_json(P("banana", b"green_from_run2")),
                           op_json(D("cherry"))]},
    })
    # decode errors, hand-derived from runs.rs:537-624 (check order per record)
    good = fmt.encode_record(P("k", b"v"))
    dec = [
        ("empty", b"", "EmptyInput", "Input list of operations cannot be empty", 0),
        ("version2", bytes([2, 0]), "UnsupportedVersion", "Unsupported run version: 2", 0),
        ("keylen_eof", b"\x01" + good + b"\x01\x00\x00", "Io", "I/O error: failed to fill whole buffer", 1),
        ("key_incomplete", b"\x01" + good + b"\x01\x00\x00\x00\x09abc", "Format",
         "Data format error: Incomplete key data", 1),
        ("bad_utf8", b"\x01" + good + b"\x02\x00\x00\x00\x02\xc3\x28", "Format",
         "Data format error: Invalid UTF-8 in key", 1),
        ("vallen_eof", b"\x01" + good + b"\x01\x00\x00\x00\x01k\x00", "Io", "I/O error: failed to fill whole buffer", 1),
        ("val_incomplete", b"\x01" + good + b"\x01\x00\x00\x00\x01k\x00\x00\x00\x05ab", "Format",
         "Data format error: Incomplete value data", 1),
        ("bad_marker", b"\x01" + good + b"\x07\x00\x00\x00\x01k", "Format", "Data format error: Invalid marker byte: 7", 1),
        # the key is read (and UTF-8 checked) before the marker is matched (runs.rs:579-595)
        ("bad_marker_after_bad_utf8", b"\x01\x07\x00\x00\x00\x01\xff", "Format",
         "Data format error: Invalid UTF-8 in key", 0),
        ("delete_then_eof_ok", b"\x01" + fmt.encode_record(D("z")), None, None, 1),
        ("version_only_ok", b"\x01", None, None, 0),
    ]
    for name, data, err, msg, n in dec:
        k.append({"name": "decode_" + name, "ref": "src/runs.rs:517-628 (hand-derived)", "kind": "decode",
                  "hex": h(data), "expect": {"n_ops": n, "error": err, "message": msg}})
    return k


def run_list_json(runs):
    return [{"hex": h(b), "min_key": h(st[0]), "max_key": h(st[1]), "size_bytes": st[2], "put_count": st[3],
             "delete_count": st[4], "table_id": t} for b, st, t in runs]


def compact_cases():
    import pyoracle

    cases = []

    def add(name, streams, max_size, flags=0, note=""):
        try:
            ref_runs, ref_dropped = pyref.compact(streams, max_size, flags)
            ref = {"runs": run_list_json(ref_runs), "dropped_tables": ref_dropped}
        except pyref.Err as e:
            ref = {"error_code": e.code, "message": e.msg}
        try:
            runs, info = pyoracle.compact(streams, max_size, flags, with_result=True)
            ora = {"runs": [{"hex": h(r.data), "min_key": h(r.stats.min_key.encode()),
                             "max_key": h(r.stats.max_key.encode()), "size_bytes": r.stats.size_bytes,
                             "put_count": r.stats.put_count, "delete_count": r.stats.delete_count,
                             "table_id": r.table_id} for r in runs],
                   "dropped_tables": info["dropped_tables"]}
        except Exception as e:  # RunError
            ora = {"error_code": e.code, "message": e.message}
        assert ora == ref, f"{name}: oracle and pyref disagree\n{ora}\n{ref}"
        blob = b"".join(bytes.fromhex(r["hex"]) for r in ora.get("runs", []))
        cases.append({"name": name, "note": note, "max": max_size, "flags": flags,
                      "streams": [[s, [h(r) for r in runs]] for s, runs in streams],
                      "expect": ora, "sha256": hashlib.sha256(blob).hexdigest()})

    P, D, enc = fmt.put, fmt.delete, fmt.encode_run
    add("two_way_overlap", [(1, [enc([P("a", b"1"), P("c", b"3")])]), (2, [enc([P("a", b"10"), P("b", b"20")])])], 4 * MiB)
    add("tombstones_kept", [(5, [enc([P("a", b"x"), D("b"), P("d", b"dd")])]),
                            (3, [enc([P("b", b"old"), P("c", b"c"), D("d")])])], 4 * MiB)
    add("tombstones_dropped", [(5, [enc([P("a", b"x"), D("b"), P("d", b"dd")])]),
                               (3, [enc([P("b", b"old"), P("c", b"c"), D("d")])])], 4 * MiB, 1)
    add("all_deleted_dropped", [(2, [enc([D("a"), D("b")])]), (1, [enc([P("a", b"1"), P("b", b"2")])])], 4 * MiB, 1)
    add("l0_concat_stream", [(7, [enc([P("m", b"new")])]),
                             (0, [enc([P("a", b"1"), P("f", b"2")]), enc([P("k", b"3"), P("m", b"old")]),
                                  enc([P("x", b"4")])])], 4 * MiB, 0, "buffer run + L0 runs concatenated at SeqNo 0")
    add("empty_stream_skipped", [(1, []), (2, [enc([P("q", b"1")])])], 4 * MiB)
    add("nothing", [], 4 * MiB)
    add("version_only_runs", [(1, [b"\x01"]), (2, [b"\x01", b"\x01"])], 4 * MiB)
    add("split_small_max", [(1, [enc([P(f"k{i:03d}", bytes([i]) * (i % 7)) for i in range(60)])])], 64)
    add("split_max_zero", [(1, [enc([P("a", b"1"), D("b"), P("c", b"")])])], 0)
    add("oversized_record", [(1, [enc([P("a", b"x" * 100), P("b", b"y"), P("c", b"z" * 200)])])], 50)
    add("long_shared_prefix", [(2, [enc([P("p" * 40 + "a", b"1"), P("p" * 40 + "c", b"3")])]),
                               (1, [enc([P("p" * 17, b"short"), P("p" * 40 + "a", b"old"),
                                         P("p" * 40 + "b", b"2")])])], 4 * MiB, 0, "keys > 16 B sharing a 40 B prefix")
    add("prefix_keys", [(1, [enc([P("ab", b"1"), P("abc", b"2"), P("abcdefghijklmnop", b"3"),
                                  P("abcdefghijklmnopq", b"4")])]), (2, [enc([P("abc", b"N")])])], 4 * MiB)
    add("utf8_keys", [(1, [enc([P("café", b"1"), P("日本", b"2"), P("\U0001f600", b"3")])]),
                      (2, [enc([P("café", b"x")])])], 4 * MiB)
    add("empty_key_and_value", [(1, [enc([P("", b""), P("a", b"")])]), (2, [enc([D("")])])], 4 * MiB)
    add("in_stream_dup_dropped", [(1, [enc([P("a", b"first"), P("a", b"second"), P("b", b"b")])])], 4 * MiB, 0,
        "a duplicate inside one stream is silently dropped by the merge (k_way.rs:146)")
    add("in_stream_decrease", [(1, [enc([P("b", b"1"), P("a", b"2")])])], 4 * MiB, 0,
        "a key decrease inside a stream trips build_runs' order check (runs.rs:190-198)")
    add("decrease_vs_decode_error_order",
        [(2, [enc([P("a", b"1"), P("m", b"2"), P("c", b"3")])]), (1, [enc([P("b", b"1")]) + b"\x09"])], 4 * MiB, 0,
        "stream 1 errors after 'b'; stream 2 decreases after 'm' (pops later) -> the decode error wins")
    add("decode_error_vs_decrease_order",
        [(2, [enc([P("a", b"1"), P("c", b"2"), P("b", b"3")])]), (1, [enc([P("x", b"1")]) + b"\x09"])], 4 * MiB, 0,
        "stream 2 decreases after 'c', which pops before stream 1's 'x' -> the order error wins")
    add("init_error_vector_order", [(1, [enc([P("a", b"1")])]), (2, [b""]), (3, [b"\x05"])], 4 * MiB, 0,
        "first items are pulled in vector order (k_way.rs:126-140): stream 2's EmptyInput wins")
    add("error_in_second_member", [(1, [enc([P("a", b"1")]), b"\x02\x00"]), (2, [enc([P("b", b"1")])])], 4 * MiB)
    add("bad_marker_stream", [(1, [enc([P("a", b"1"), P("c", b"3")])]), (2, [enc([P("b", b"1")]) + b"\x03\x00\x00\x00\x00"])],
        4 * MiB)
    add("wal_two_tables", [(1, [enc([P("1.a", b"x"), P("1.b", b"y"), P("2.a", b"z")])]),
                           (2, [enc([D("1.a"), P("2.c", b"w")])])], 4 * MiB, 2)
    add("wal_negative_and_prefix_quirks", [(1, [enc([P("+5.a", b"1"), P("-0.b", b"2"), P("007.c", b"3"), P("7.d", b"4")])])],
        4 * MiB, 2, "format!(\"{id}.\").len() strip quirk (wal_compaction.rs:81)")
    add("wal_table_too_big_dropped", [(1, [enc([P(f"3.k{i:02d}", b"v" * 30) for i in range(10)] +
                                               [P("4.a", b"1")])])], 200, 2,
        "table 3 needs > 1 run -> its task errors and is swallowed (wal_compaction.rs:131-137, :103)")
    add("wal_bad_key", [(1, [enc([P("1.a", b"x"), P("nodot", b"y")])])], 4 * MiB, 2)
    add("wal_bad_table_id", [(1, [enc([P("1.a", b"x"), P("1x.b", b"y")])])], 4 * MiB, 2)
    add("wal_table_overflow", [(1, [enc([P("99999999999999999999.a", b"x")])])], 4 * MiB, 2)
    add("wal_empty_prefix", [(1, [enc([P(".a", b"x")])])], 4 * MiB, 2)
    # generated shapes (scaled-down configs)
    add("cfg1_scaled", gen.config1(n_records=300), 4 * MiB)
    add("cfg2A_scaled_small_max", gen.config2(n_streams=8, n_records=120, vsize=32), 2048)
    add("cfg2B_scaled", gen.config2(n_streams=6, n_records=150, vsize=16, variant="B"), 4096)
    add("cfg3_scaled", gen.config3(n_streams=5, run_bytes=20 * KiB, vsize=24), 8 * KiB)
    add("cfg3_scaled_drop", gen.config3(n_streams=5, run_bytes=20 * KiB, vsize=24), 8 * KiB, 1)
    add("cfg5_scaled", gen.config5(n_streams=40, n_records=12), 4 * MiB, 2)
    return cases


def main():
    k = kats()
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(k, f, indent=1)
    c = compact_cases()
    with open(os.path.join(HERE, "compact_cases.json"), "w") as f:
        json.dump(c, f, indent=0)
    print(f"wrote {len(k)} KATs and {len(c)} compaction cases")


if __name__ == "__main__":
    main()
