"""The compaction jobs' input-stream assembly (src/jobs/*.rs), minus storage and metadata.

Each function builds exactly the (SeqNo, stream) list the reference job hands to
k_way::merge and runs it through the device path. The caller supplies run bytes instead of
RunIDs (the jobs' get_run/put_run and append_* commits stay on the skyvault side).
"""
from __future__ import annotations

from typing import Dict, List, Sequence

from ._abi import SKV_DROP_TOMBSTONES, SKV_SPLIT_BY_TABLE, OutRun
from .api import MAX_RUN_SIZE, Compactor

FAN_IN_CAP = 16  # table_buffer_compaction.rs:32, wal_compaction.rs:18
LEVEL_MAX = 6    # metadata.rs:117-126


def table_buffer_compaction(c: Compactor, buffer: Dict[int, bytes], level0: Sequence[bytes],
                            max_run_size: int = MAX_RUN_SIZE) -> List[OutRun]:
    """table_buffer_compaction.rs:32-103: the oldest min(16, n) buffer runs, each at its own
    SeqNo (BTreeMap order), plus every L0 run concatenated (min_key order) as ONE stream at
    SeqNo 0 when the table has a level 0 (:243-276). Output runs belong to L0."""
    streams = [(seq, [data]) for seq, data in sorted(buffer.items())[:FAN_IN_CAP]]
    if level0 is not None:
        streams.append((0, list(level0)))
    return c.compact(streams, max_run_size, 0)


def table_tree_compaction(c: Compactor, level_run: bytes, next_level_runs: Sequence[bytes], level: int,
                          max_run_size: int = MAX_RUN_SIZE) -> List[OutRun]:
    """table_tree_compaction.rs:81-147: the chosen level-L run at SeqNo 1 against the
    overlapping level-L+1 runs concatenated at SeqNo 0; Deletes are dropped when L+1 is
    Level::max() (:139-145)."""
    if level >= LEVEL_MAX:
        return []
    flags = SKV_DROP_TOMBSTONES if level + 1 == LEVEL_MAX else 0
    return c.compact([(1, [level_run]), (0, list(next_level_runs))], max_run_size, flags)


def wal_compaction(c: Compactor, wal: Dict[int, bytes], max_run_size: int = MAX_RUN_SIZE) -> List[OutRun]:
    """wal_compaction.rs:18-174: the oldest min(16, n) WAL runs at their own SeqNos, merged,
    split by "{table_id}." key prefix into one run per table (OutRun.table_id)."""
    streams = [(seq, [data]) for seq, data in sorted(wal.items())[:FAN_IN_CAP]]
    return c.compact(streams, max_run_size, SKV_SPLIT_BY_TABLE)
