#!/bin/bash
# Round-6 first GPU call: the default bench line on this round's code, and config 3F under the
# per-dispatch kernel trace (which k_tile<true> launch is the slow one).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r06/p1"; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > "$O/bench_default.log" 2>&1 || { echo "bench rc=$?"; tail -5 "$O/bench_default.log"; exit 1; }
grep -E '^\{"metric"' "$O/bench_default.log" | tail -1
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$O/trace3F" -o run -- \
  python3 "$R/bench.py" --config 3F --steps 5 --warmup 1 --no-host-path --no-cpu-baseline > "$O/bench_3F.log" 2>&1
rc=$?; cd "$R"; [ $rc -ne 0 ] && { echo "3F rc=$rc"; tail -5 "$O/bench_3F.log"; exit 1; }
grep -E '^\{"metric"' "$O/bench_3F.log" | tail -1 | cut -c1-400
f=$(find "$O/trace3F" -name "*kernel_trace.csv" | head -1)
python3 tools/r06/dispatch.py "$f" 1 5 --dispatches 'k_tile<true>' --out "$O/kstats_3F.csv" > "$O/kstats_3F.txt"
cat "$O/kstats_3F.txt" | head -60
rm -rf "$O/trace3F"
