#!/bin/bash
# PMC counter passes (one rocprofv3 --pmc run per counter group, kernel-trace only, no sys/hip
# trace domains). Output CSVs under gpurun_out/pmc/<group>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/pmc"
export TMPDIR=/tmp
cd /tmp
if [ "${LIST:-0}" = "1" ]; then rocprofv3 -L > "$R/gpurun_out/pmc/counters_list.txt" 2>&1 || true; fi
i=0
for grp in ${PMC_GROUPS:-FETCH_SIZE WRITE_SIZE}; do
  grp=${grp//,/ }
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/pmc/g$i" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$R/gpurun_out/pmc/g$i.log" 2>&1
  rc=$?; echo "pmc group $i ($grp) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
