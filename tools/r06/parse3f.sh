#!/bin/bash
# staged chunk walks (the parse reads the input once): parity on the general path, config 3 at full
# size, then the 3F bench under the kernel trace (timed dispatches)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r06/p3f"; mkdir -p "$O"
export TMPDIR=/tmp
if [ "${PARITY:-1}" = 1 ]; then
  timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_split.py tests/test_gpu_shard_split.py \
    tests/test_gpu_hostpipe.py tests/test_gpu_search.py tests/test_gpu_scan.py ${EXTRA_TESTS:-} > "$O/pytest.log" 2>&1
  rc=$?; tail -4 "$O/pytest.log"; [ $rc -ne 0 ] && exit 1
fi
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$O/t3F" -o run -- \
  python3 "$R/bench.py" --config 3F --steps 3 --warmup 1 --no-host-path --no-cpu-baseline > "$O/bench_3F.log" 2>&1
rc=$?; cd "$R"; [ $rc -ne 0 ] && { echo "3F rc=$rc"; tail -5 "$O/bench_3F.log"; exit 1; }
grep -E '^\{"metric"' "$O/bench_3F.log" | tail -1 | grep -o '"ms_per_step": [0-9.]*\|"phases_ms": {[^}]*}'
f=$(find "$O/t3F" -name "*kernel_trace.csv" | head -1)
python3 tools/r06/dispatch.py "$f" 1 3 --out "$O/kstats_3F.csv" > "$O/kstats_3F.txt"
head -12 "$O/kstats_3F.txt"
rm -rf "$O/t3F"
