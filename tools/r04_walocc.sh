#!/bin/bash
# k_wal_fused occupancy A/B (SKV_WAL_LDS pads its LDS request: 7 / 4 / 3 / 2 workgroups per CU) on
# config 5: fewer record lines in flight per XCD, so the composition's re-read may hit L2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="$PWD/gpurun_out/r04"
mkdir -p "$O"
for pad in ${PADS:-0 29000 42000 69000}; do
  SKV_WAL_LDS=$pad timeout -k 10 300 python bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline --no-host-path \
    > "$O/walocc_$pad.log" 2>&1 || { echo "pad $pad failed"; tail -5 "$O/walocc_$pad.log"; exit 1; }
  echo "pad $pad $(grep -o '"ms_per_step": [0-9.]*' $O/walocc_$pad.log) $(grep -o '"phases_ms": {[^}]*' $O/walocc_$pad.log)"
done
