#!/bin/bash
# Round-4 measurement set on one MI355X, per BASELINE config (2A 2B 3 3F 5 by default, CONFIGS=...):
#   bench  the bench line (cpu_baseline included; host_path for 2A / 2B / 3)
#   prof   rocprofv3 --kernel-trace --stats of the same workload
#   pmc    FETCH_SIZE and WRITE_SIZE passes (separate runs, kernel-trace only) -> tools/traffic.py
#          keys them by config into gpurun_out/r04f/traffic.json (copy to profiles/traffic_latest.json)
# Output: gpurun_out/r04f/. STAGE=bench|prof|pmc (default: all three).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
O="$R/gpurun_out/r04f"
mkdir -p "$O"
export TMPDIR=/tmp
S="${STAGE:-bench pmc}"
CS="${CONFIGS:-2A 2B 3 3F 5 L0}"
for C in $CS; do
  if [[ " $S " == *" bench "* ]]; then
    # the bench line under rocprofv3 --kernel-trace --stats: its roofline (HIP-event launch time) and
    # the committed kernel stats come from the same process (no host-path / 2-ctx calls in it, so
    # every skv launch in the trace is one of the bench's compactions: warm-up + steps + the check)
    if [ "$C" = 2A ]; then A="--steps 20 --warmup 5"; N=26; else A="--config $C --steps 5 --warmup 1"; N=7; fi
    cd /tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/bprof_$C" -o run -- \
      python3 "$R/bench.py" $A --no-host-path > "$O/bench_$C.log" 2>&1 || { echo "bench $C failed"; tail -5 "$O/bench_$C.log"; exit 1; }
    cd "$R"
    python3 tools/kstats_skv.py "$(ls $O/bprof_$C/*kernel_stats.csv | head -1)" $N "$O/kernel_stats_$C.csv" > /dev/null
    cp "$(ls $O/bprof_$C/*kernel_stats.csv | head -1)" "$O/rocprof_stats_$C.csv"
    rm -rf "$O/bprof_$C"
    echo "bench $C: $(tail -1 $O/bench_$C.log | cut -c1-300)"
    if [ "$C" != 3F ] && [ "${HOST:-1}" = 1 ]; then  # the PCIe-inclusive figure, its own run
      timeout -k 10 600 python3 bench.py $A --no-cpu-baseline > "$O/host_$C.log" 2>&1 || { echo "host $C failed"; tail -5 "$O/host_$C.log"; exit 1; }
      echo "host $C: $(tail -1 $O/host_$C.log | grep -o '"host_path": {[^}]*' | cut -c1-200)"
    fi
  fi
  if [[ " $S " == *" prof "* ]]; then
    cd /tmp
    timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$C" -o run -- \
      python3 "$R/bench.py" --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > "$O/prof_$C.log" 2>&1 \
      || { echo "prof $C failed"; exit 1; }
    cd "$R"
    python3 tools/kstats_skv.py "$(ls $O/prof_$C/*kernel_stats.csv | head -1)" 5 "$O/kernel_stats_$C.csv" > /dev/null
    cp "$(ls $O/prof_$C/*kernel_stats.csv | head -1)" "$O/rocprof_stats_$C.csv"
    rm -rf "$O/prof_$C"  # the raw traces exceed what a call may copy back (64 MiB)
    echo "prof $C done"
  fi
  if [[ " $S " == *" pmc "* ]]; then
    i=0
    for grp in FETCH_SIZE WRITE_SIZE; do
      i=$((i+1))
      cd /tmp
      timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d "$O/pmc_$C/g$i" -o run -- \
        python3 "$R/bench.py" --config $C --steps 1 --warmup 1 --no-cpu-baseline --no-host-path > "$O/pmc_${C}_g$i.log" 2>&1 \
        || { echo "pmc $C $grp failed"; exit 1; }
      cd "$R"
    done
    python3 tools/traffic.py "$O/pmc_$C" "$C" "$O/traffic.json" > "$O/traffic_$C.txt" || { echo "traffic $C failed"; exit 1; }
    head -6 "$O/traffic_$C.txt"  # (a pipe into head broke traffic.py's output before it wrote the file)
    rm -rf "$O/pmc_$C"
    echo "pmc $C done"
  fi
done
exit 0
