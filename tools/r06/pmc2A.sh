#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of the 2A bench (one step): per-kernel traffic (tools/traffic.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r06/${TAG:-pmc2A}"; mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d "$O/pmc/$ctr" -o run -- \
    python3 "$R/bench.py" --config ${CONFIG:-2A} --steps 1 --warmup 1 --no-cpu-baseline --no-host-path > "$O/pmc_$ctr.log" 2>&1 \
    || { echo "pmc $ctr failed"; tail -3 "$O/pmc_$ctr.log"; exit 1; }
done
cd "$R"
python3 tools/traffic.py "$O/pmc" ${CONFIG:-2A} "$O/traffic.json" > "$O/traffic.txt"; head -5 "$O/traffic.txt"
rm -rf "$O/pmc"
