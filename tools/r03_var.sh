#!/bin/bash
# Run-to-run variance of the config-2A step (the round-2 "check" phase swing, 0.26 vs 0.62 ms):
# N separate bench processes on one box, each printing ms per step, the splitter ("check") phase,
# the k_fx_tile launch and the library's per-phase means; then one kernel-trace run per process
# pair so a slow run's kernels can be compared with a fast one's. Output: gpurun_out/r03/var/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
O="$R/gpurun_out/r03/var"
mkdir -p "$O"
export TMPDIR=/tmp
for i in $(seq 1 ${N:-5}); do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > "$O/b$i.log" 2>&1 \
    || { echo "bench $i failed"; tail -5 "$O/b$i.log"; exit 1; }
  echo "run $i $(grep -o '"ms_per_step": [0-9.]*' $O/b$i.log) $(grep -o '"check": [0-9.]*' $O/b$i.log) $(grep -o '"avg_launch_ms": [0-9.]*' $O/b$i.log)"
done
if [ "${PROF:-1}" = "1" ]; then
  for i in 1 2 3; do
    cd /tmp
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof$i" -o run -- \
      python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > "$O/prof$i.log" 2>&1 \
      || { echo "prof $i failed"; exit 1; }
    cd "$R"
    echo "prof $i $(grep -o '"ms_per_step": [0-9.]*' $O/prof$i.log) $(grep -o '"check": [0-9.]*' $O/prof$i.log)"
  done
fi
exit 0
