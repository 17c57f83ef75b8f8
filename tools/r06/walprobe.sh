#!/bin/bash
# config 5: k_wal_fused phase knockouts (SKV_WAL_PROBE builds, output invalid: --no-check) and the
# product, timed dispatches of k_wal_fused per variant (VARIANTS="base wp1 wp2", base = libskv.so;
# build wpN with: make -C skyvault-rs_amd variant TAG=wpN VFLAGS=-DSKV_WAL_PROBE=N)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r06/wal"; mkdir -p "$O"
export TMPDIR=/tmp
if [ "${PARITY:-1}" = 1 ]; then
  timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_sort.py tests/test_gpu_split.py tests/test_gpu_shard_split.py \
    tests/test_gpu_hostpipe.py "tests/test_gpu_fullsize.py::test_config5_full_size" > "$O/pytest.log" 2>&1
  rc=$?; tail -4 "$O/pytest.log"; [ $rc -ne 0 ] && exit 1
fi
for v in ${VARIANTS:-base wp1 wp2}; do
  lib="$R/skyvault-rs_amd/skv/libskv.so"; chk=""
  [ "$v" != base ] && lib="$R/skyvault-rs_amd/skv/variants/libskv_$v.so"
  case $v in wp*) chk="--no-check";; esac
  cd /tmp
  SKV_LIB="$lib" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/t_$v" -o run -- \
    python3 "$R/bench.py" --config 5 --steps 6 --warmup 2 --no-host-path --no-cpu-baseline $chk > "$O/bench_$v.log" 2>&1
  rc=$?; cd "$R"; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 "$O/bench_$v.log"; exit 1; }
  echo "== $v $(grep -E '^\{"metric"' "$O/bench_$v.log" | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
  f=$(find "$O/t_$v" -name "*kernel_trace.csv" | head -1)
  python3 tools/r06/dispatch.py "$f" 2 6 --out "$O/kstats_$v.csv" > "$O/kstats_$v.txt"
  grep -E "wal_fused|sort_tile|total" "$O/kstats_$v.txt" | head -4
  rm -rf "$O/t_$v"
done
