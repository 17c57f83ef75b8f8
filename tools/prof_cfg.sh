#!/bin/bash
# rocprofv3 kernel-trace summary of bench.py --config C (steps 3, warmup 1) for each C given.
# Output: gpurun_out/pc_<C>/run_kernel_stats.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in "$@"; do
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pc_$C" -o run -- \
    python3 "$R/bench.py" --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > "$R/gpurun_out/pc_$C.log" 2>&1 \
    || { echo "prof $C failed"; exit 1; }
  cd "$R"
  echo "prof $C done"
done
