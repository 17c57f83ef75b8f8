#!/bin/bash
# Round-6 measurement record on one MI355X: for each config, the bench line (no profiler), the same
# timed loop under rocprofv3 --kernel-trace with per-kernel stats of the TIMED calls only
# (tools/r06/dispatch.py drops warm-ups and the check call), then two PMC passes (FETCH_SIZE,
# WRITE_SIZE; kernel trace only) for the per-launch and per-call traffic (tools/traffic.py).
# CONFIGS="2A 2B 3 3F 5 L0"; PMC=0 skips the counters. Output: gpurun_out/r06/final/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r06/final"; mkdir -p "$O"
export TMPDIR=/tmp
for c in ${CONFIGS:-2A 2B 3 3F 5 L0}; do
  W=3; K=${STEPS:-20}; extra=""
  if [ "${BENCH:-1}" = 1 ]; then
  [ "$c" = 3F ] && { W=1; K=5; extra="--no-host-path"; }
  [ "$c" = 5 ] && { W=2; K=10; }
  timeout -k 10 600 python3 bench.py --config $c --steps $K --warmup $W $extra > "$O/bench_$c.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "bench $c rc=$rc"; tail -5 "$O/bench_$c.log"; exit $rc; }
  grep -E '^\{"metric"' "$O/bench_$c.log" | tail -1 > "$O/bench_$c.json"
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_$c" -o run -- \
    python3 "$R/bench.py" --config $c --steps $K --warmup $W --no-host-path --no-cpu-baseline > "$O/bench_prof_$c.log" 2>&1
  rc=$?; cd "$R"
  [ $rc -ne 0 ] && { echo "prof $c rc=$rc"; tail -5 "$O/bench_prof_$c.log"; exit $rc; }
  grep -E '^\{"metric"' "$O/bench_prof_$c.log" | tail -1 > "$O/bench_prof_$c.json"
  f=$(find "$O/trace_$c" -name "*kernel_trace.csv" | head -1)
  python3 tools/r06/dispatch.py "$f" $W $K --out "$O/kernel_stats_$c.csv" > "$O/kernel_stats_$c.txt"
  f=$(find "$O/trace_$c" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$O/rocprof_stats_$c.csv"
  sed -n 1,6p "$O/kernel_stats_$c.txt"
  echo "$c: $(grep -o '"value": [0-9.]*' $O/bench_$c.json | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$c.json)"
  fi
  if [ "${PMC:-1}" = 1 ]; then
    pe="--steps 1 --warmup 1 --no-cpu-baseline --no-host-path"
    for ctr in FETCH_SIZE WRITE_SIZE; do
      cd /tmp
      timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d "$O/pmc_$c/$ctr" -o run -- \
        python3 "$R/bench.py" --config $c $pe > "$O/pmc_${c}_$ctr.log" 2>&1
      rc=$?; cd "$R"; [ $rc -ne 0 ] && { echo "pmc $c $ctr rc=$rc"; tail -3 "$O/pmc_${c}_$ctr.log"; exit $rc; }
    done
    # (one traffic file per config: a call's gpurun_out merge must not replace another call's)
    python3 tools/traffic.py "$O/pmc_$c" $c "$O/traffic_$c.json" 3 > "$O/traffic_$c.txt"
    sed -n 1,3p "$O/traffic_$c.txt"
  fi
  [ "${KEEP_TRACES:-0}" = 1 ] || rm -rf "$O/trace_$c" "$O/pmc_$c"
done
