#!/bin/bash
# config 5 bench under the kernel trace (timed dispatches), optional parity subset first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r06/c5"; mkdir -p "$O"
export TMPDIR=/tmp
if [ "${PARITY:-0}" = 1 ]; then
  timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_sort.py tests/test_gpu_fused.py tests/test_gpu_hostpipe.py \
    ${EXTRA_TESTS:-} > "$O/pytest.log" 2>&1
  rc=$?; tail -3 "$O/pytest.log"; [ $rc -ne 0 ] && exit 1
fi
for v in ${VARIANTS:-base}; do
  lib="$R/skyvault-rs_amd/skv/variants/libskv_$v.so"; [ "$v" = base ] && lib="$R/skyvault-rs_amd/skv/libskv.so"
  cd /tmp
  SKV_LIB="$lib" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/t_$v" -o run -- \
    python3 "$R/bench.py" --config 5 --steps 6 --warmup 2 --no-host-path --no-cpu-baseline > "$O/bench_$v.log" 2>&1
  rc=$?; cd "$R"; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 "$O/bench_$v.log"; exit 1; }
  echo "== $v $(grep -E '^\{"metric"' "$O/bench_$v.log" | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
  f=$(find "$O/t_$v" -name "*kernel_trace.csv" | head -1)
  python3 tools/r06/dispatch.py "$f" 2 6 --out "$O/kstats_$v.csv" > "$O/kstats_$v.txt"
  head -12 "$O/kstats_$v.txt" | tail -10
  rm -rf "$O/t_$v"
done
