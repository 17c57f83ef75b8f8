"""skv — MI355X-native compaction path for skyvault v1 runs.

The product is libskv.so (HIP kernels for gfx950 behind the C ABI in include/skv.h).
This package is its host-side mirror of the reference interface:

  skv.api.Compactor.compact(...)   read_run_stream -> k_way::merge -> [filter] -> build_runs
  skv.jobs.*                       the compaction jobs' input-stream assembly (src/jobs/*.rs)
  skv.format                       the v1 run format (runs.rs:97-100, :240-267)
  skv.gen                          deterministic synthetic workloads (BASELINE.json configs)
"""
from ._abi import (  # noqa: F401
    SKV_DROP_TOMBSTONES,
    SKV_SPLIT_BY_TABLE,
    OutRun,
    RunError,
    Stats,
)
