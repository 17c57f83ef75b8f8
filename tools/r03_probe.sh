#!/bin/bash
# fetch_probe under rocprofv3: timings, then separate --pmc passes (kernel-trace only) for
# FETCH_SIZE, and the TCC read-request counters. Output: gpurun_out/r03/probe/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
O="$R/gpurun_out/r03/probe"
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 60 "$R/tools/ubench/fetch_probe" > "$O/times.txt" 2>&1 || { cat "$O/times.txt"; exit 1; }
cat "$O/times.txt"
cd /tmp
i=0
for grp in FETCH_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$O/g$i" -o run -- "$R/tools/ubench/fetch_probe" \
    > "$O/g$i.log" 2>&1 || { echo "pmc $grp failed"; tail -5 "$O/g$i.log"; exit 1; }
  echo "pmc $grp done"
done
exit 0
