#!/bin/bash
# k_fx_tile phase ticks (SKV_TILE_PROF build) and the 2A per-dispatch trace of the timed steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r06/p6"; mkdir -p "$O"
export TMPDIR=/tmp
SKV_LIB=$R/skyvault-rs_amd/skv/variants/libskv_tprof.so timeout -k 10 300 python3 tools/r06/tileprof.py 16 2A 2>&1 | grep -E "call|tile phase" || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/trace2A" -o run -- \
  python3 "$R/bench.py" --steps 10 --warmup 2 --no-host-path --no-cpu-baseline > "$O/bench_2A.log" 2>&1
rc=$?; cd "$R"; [ $rc -ne 0 ] && { echo "2A rc=$rc"; tail -5 "$O/bench_2A.log"; exit 1; }
grep -E '^\{"metric"' "$O/bench_2A.log" | tail -1 | cut -c1-250
f=$(find "$O/trace2A" -name "*kernel_trace.csv" | head -1)
python3 tools/r06/dispatch.py "$f" 2 10 --out "$O/kstats_2A.csv" > "$O/kstats_2A.txt"
cat "$O/kstats_2A.txt"
python3 - "$f" <<'PY'
import csv, sys
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in csv.DictReader(open(sys.argv[1])) if "skv::" in r["Kernel_Name"])
# one timed compaction's timeline: the 5th k_run_header onwards
starts = [i for i, r in enumerate(rows) if "k_run_header" in r[2]]
a = starts[5]; b = starts[6]
t0 = rows[a][0]
for s, e, n in rows[a:b]:
    print(f"{(s - t0) / 1e3:9.1f} us +{(e - s) / 1e3:8.1f} us  {n}")
PY
rm -rf "$O/trace2A"
