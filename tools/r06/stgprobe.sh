#!/bin/bash
# 3F variants (SKV_LIB builds; base = libskv.so; --no-check), timed dispatches of the parse kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r06/stg"; mkdir -p "$O"
export TMPDIR=/tmp
for v in ${VARIANTS:-sp1 sp2 sp3}; do
  cd /tmp
  lib="$R/skyvault-rs_amd/skv/variants/libskv_$v.so"; [ "$v" = base ] && lib="$R/skyvault-rs_amd/skv/libskv.so"
  SKV_LIB="$lib" timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv \
    -d "$O/t_$v" -o run -- python3 "$R/bench.py" --config 3F --steps 2 --warmup 1 --no-host-path --no-cpu-baseline --no-check \
    > "$O/bench_$v.log" 2>&1
  rc=$?; cd "$R"; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 "$O/bench_$v.log"; exit 1; }
  f=$(find "$O/t_$v" -name "*kernel_trace.csv" | head -1)
  python3 tools/r06/dispatch.py "$f" 1 2 > "$O/kstats_$v.txt"
  echo "== $v"; grep -E "${PAT:-k_spec|k_emit}" "$O/kstats_$v.txt"
  rm -rf "$O/t_$v"
done
