#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r06/p3"; mkdir -p "$O"
for v in tprof tprof_old; do
  echo "== $v"
  SKV_LIB=$R/skyvault-rs_amd/skv/variants/libskv_$v.so timeout -k 10 300 python3 tools/r06/tileprof.py 16 > "$O/$v.log" 2>&1 || { tail -5 "$O/$v.log"; exit 1; }
  cat "$O/$v.log" | grep -v "^ "
done
