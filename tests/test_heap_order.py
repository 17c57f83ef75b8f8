"""k_way::merge's pop order for UNSORTED streams (the basis of skv_heap.hip's heap-order mode):
a literal binary-heap merge (tests/pyref.py, k_way.rs:113-179) pops records in the stable order
of (running maximum of the stream's keys up to the record, seq_no descending, position)."""
import random

import pyref
from skv import format as fmt


def _e_order(streams):
    items = []
    for seq, ops in streams:
        m = None
        for p, op in enumerate(ops):
            m = op[1] if m is None or op[1] > m else m
            items.append(((m, -seq, p), op))
    items.sort(key=lambda x: x[0])
    out, last = [], None
    for _, op in items:  # first per key among consecutive pops (k_way.rs:146-151)
        if last is None or op[1] != last:
            out.append(op)
        last = op[1]
    return out


def test_prefix_max_order_equals_heap_pops():
    r = random.Random(5)
    for _ in range(3000):
        streams = []
        for seq in r.sample(range(-20, 100), r.randint(1, 6)):
            keys = [bytes([97 + r.randrange(8)]) * r.randint(1, 2) for _ in range(r.randint(0, 8))]
            ops = [fmt.put(k.decode(), b"%d" % seq) if r.random() < 0.7 else fmt.delete(k.decode()) for k in keys]
            streams.append((seq, ops))
        runs = [(seq, [fmt.encode_run(ops)]) for seq, ops in streams]
        heap = list(pyref.merge(runs))
        exp = [(o[1], o[2]) for o in _e_order(streams)]
        assert [(key, v) for _, key, v in heap] == exp
