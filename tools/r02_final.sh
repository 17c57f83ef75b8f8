#!/bin/bash
# Round-2 measurement set on one MI355X: the bench line of every BASELINE config (cpu_baseline
# included), a rocprofv3 kernel-trace summary per config, and the FETCH_SIZE / WRITE_SIZE PMC
# passes of the headline config (separate runs, kernel-trace only). Output: gpurun_out/r02f/.
# STAGE=bench|prof|pmc (default: all three).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
O="$R/gpurun_out/r02f"
mkdir -p "$O"
export TMPDIR=/tmp
S="${STAGE:-bench prof pmc}"
if [[ " $S " == *" bench "* ]]; then
  timeout -k 10 420 python3 bench.py > "$O/bench_2A.log" 2>&1 || { echo "bench 2A failed"; exit 1; }
  echo "bench 2A done"
  for C in 2B 3 3F 5; do
    timeout -k 10 420 python3 bench.py --config $C --steps 3 --warmup 1 --no-host-path > "$O/bench_$C.log" 2>&1 \
      || { echo "bench $C failed"; exit 1; }
    echo "bench $C done"
  done
fi
if [[ " $S " == *" prof "* ]]; then
  for C in 2A 2B 3 3F 5; do
    cd /tmp
    timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$C" -o run -- \
      python3 "$R/bench.py" --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > "$O/prof_$C.log" 2>&1 \
      || { echo "prof $C failed"; exit 1; }
    cd "$R"
    echo "prof $C done"
  done
fi
if [[ " $S " == *" pmc "* ]]; then
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    cd /tmp
    timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$O/pmc/g$i" -o run -- \
      python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-host-path > "$O/pmc_g$i.log" 2>&1 \
      || { echo "pmc $grp failed"; exit 1; }
    cd "$R"
    echo "pmc $grp done"
  done
fi
exit 0
