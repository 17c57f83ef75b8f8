#!/bin/bash
# Kernel trace + PMC passes (one counter group per run, kernel-trace only) of bench.py --config C.
# usage: pmc_counters.sh C "grp1" "grp2" ...   (a group = space-separated counters, quoted)
# Output: gpurun_out/pk_<C>/trace, gpurun_out/pk_<C>/g<i>/run_counter_collection.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
C=$1; shift
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pk_$C/trace" -o run -- \
  python3 "$R/bench.py" --config $C --steps 1 --warmup 0 --no-cpu-baseline --no-host-path > "$R/gpurun_out/pk_$C.trace.log" 2>&1 \
  || { echo "trace $C failed"; exit 1; }
echo "trace $C done"
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/pk_$C/g$i" -o run -- \
    python3 "$R/bench.py" --config $C --steps 1 --warmup 0 --no-cpu-baseline --no-host-path > "$R/gpurun_out/pk_$C.g$i.log" 2>&1 \
    || { echo "pmc $C g$i failed"; exit 1; }
  echo "pmc $C g$i ($grp) done"
done
