#!/bin/bash
# Round-5 measurement record on one MI355X: for each config, the bench line under
# rocprofv3 --kernel-trace --stats (the line and the kernel stats from the same process), then two
# PMC passes (FETCH_SIZE, WRITE_SIZE; kernel trace only) for the traffic table.
# CONFIGS="2A 2B 3 3F 5 L0"; PMC=0 skips the counters. Output: gpurun_out/r05/final/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r05/final"; mkdir -p "$O"
export TMPDIR=/tmp
for c in ${CONFIGS:-2A 2B 3 3F 5 L0}; do
  extra="--steps ${STEPS:-20} --warmup 3"
  [ "$c" = 3F ] && extra="--steps 5 --warmup 1 --no-host-path"
  [ "$c" = 5 ] && extra="--steps 10 --warmup 2"
  # the full bench line (extras included), no profiler
  timeout -k 10 600 python3 bench.py --config $c $extra > "$O/bench_$c.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "bench $c rc=$rc"; tail -5 "$O/bench_$c.log"; exit $rc; }
  grep -E '^\{"metric"' "$O/bench_$c.log" | tail -1 > "$O/bench_$c.json"
  # the same timed loop under the kernel trace, without the extras (host path, config 4, CPU
  # baseline), so the trace's dominant-kernel average is the bench line's own launches
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_$c" -o run -- \
    python3 "$R/bench.py" --config $c $extra --no-host-path --no-cpu-baseline > "$O/bench_prof_$c.log" 2>&1
  rc=$?; cd "$R"
  [ $rc -ne 0 ] && { echo "prof $c rc=$rc"; tail -5 "$O/bench_prof_$c.log"; exit $rc; }
  grep -E '^\{"metric"' "$O/bench_prof_$c.log" | tail -1 > "$O/bench_prof_$c.json"
  n=$(python3 -c "import json; d=json.load(open('$O/bench_prof_$c.json')); print(d['steps']+d['warmup']+1)")
  f=$(find "$O/trace_$c" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$O/rocprof_stats_$c.csv"
  python3 tools/kstats_skv.py "$f" $n "$O/kernel_stats_$c.csv" > "$O/kernel_stats_$c.txt"
  head -3 "$O/kernel_stats_$c.txt"
  echo "$c: $(grep -o '"value": [0-9.]*' $O/bench_$c.json | head -1) $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$c.json)"
  if [ "${PMC:-1}" = 1 ]; then
    pe="--steps 1 --warmup 1 --no-cpu-baseline --no-host-path"
    for ctr in FETCH_SIZE WRITE_SIZE; do
      cd /tmp
      timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d "$O/pmc_$c/$ctr" -o run -- \
        python3 "$R/bench.py" --config $c $pe > "$O/pmc_${c}_$ctr.log" 2>&1
      rc=$?; cd "$R"; [ $rc -ne 0 ] && { echo "pmc $c $ctr rc=$rc"; tail -3 "$O/pmc_${c}_$ctr.log"; exit $rc; }
    done
    python3 tools/traffic.py "$O/pmc_$c" $c "$O/traffic.json" > "$O/traffic_$c.txt"
    sed -n 1,3p "$O/traffic_$c.txt"
  fi
  # the per-dispatch CSVs are large (3F: past what a gpurun call brings back); the summaries stay
  [ "${KEEP_TRACES:-0}" = 1 ] || rm -rf "$O/trace_$c" "$O/pmc_$c"
done
