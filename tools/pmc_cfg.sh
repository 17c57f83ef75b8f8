#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs, kernel-trace only) of bench.py --config C.
# Output: gpurun_out/pmc_<C>/g<i>/run_counter_collection.csv (tools/traffic.py reads them).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
C=${1:-3F}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  cd /tmp
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/pmc_$C/g$i" -o run -- \
    python3 "$R/bench.py" --config $C --steps 1 --warmup 0 --no-cpu-baseline --no-host-path > "$R/gpurun_out/pmc_$C.g$i.log" 2>&1 \
    || { echo "pmc $grp failed"; exit 1; }
  cd "$R"
  echo "pmc $C $grp done"
done
