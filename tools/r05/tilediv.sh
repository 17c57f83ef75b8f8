#!/bin/bash
# Fused tiles of 1/d of the target at the same sample spacing (SKV_FX_TILE_DIV), config 2A: bench
# phases and kernel stats per d. Output: gpurun_out/r05/tilediv/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r05/tilediv"; mkdir -p "$O"
export TMPDIR=/tmp
for d in ${DIVS:-1 2 3}; do
  SKV_FX_TILE_DIV=$d timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > "$O/bench_$d.log" 2>&1 || { echo "d=$d failed"; tail -3 "$O/bench_$d.log"; exit 1; }
  echo "d=$d $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$d.log) $(grep -o '"phases_ms": {[^}]*' $O/bench_$d.log)"
done
