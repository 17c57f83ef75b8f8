#!/bin/bash
# 3F: FETCH_SIZE and WRITE_SIZE passes (kernel trace only, one counter block each) -> per-launch and
# per-call traffic (tools/traffic.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r06/pmc3f"; mkdir -p "$O"
export TMPDIR=/tmp
C=${CONFIG:-3F}
for ctr in FETCH_SIZE WRITE_SIZE; do
  cd /tmp
  timeout -s KILL 400 rocprofv3 --pmc $ctr --output-format csv -d "$O/pmc_$C/$ctr" -o run -- \
    python3 "$R/bench.py" --config $C --steps 1 --warmup 1 --no-cpu-baseline --no-host-path > "$O/pmc_${C}_$ctr.log" 2>&1
  rc=$?; cd "$R"; [ $rc -ne 0 ] && { echo "pmc $ctr rc=$rc"; tail -3 "$O/pmc_${C}_$ctr.log"; exit 1; }
done
python3 tools/traffic.py "$O/pmc_$C" $C "$O/traffic.json" 3 > "$O/traffic_$C.txt"
head -14 "$O/traffic_$C.txt"
rm -rf "$O/pmc_$C"
