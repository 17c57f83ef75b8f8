#!/bin/bash
# Record-sort bucket-search variants (tools/build_variants_r04.sh sb*) on config 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="$PWD/gpurun_out/r04"
mkdir -p "$O"
for v in ${VARIANTS:-base sbatom2 sbtop256 sbtop2048 sbper8 sbper32}; do
  lib=skyvault-rs_amd/skv/libskv.so
  [ "$v" != base ] && lib=skyvault-rs_amd/skv/variants/libskv_$v.so
  SKV_LIB=$lib timeout -k 10 300 python bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline --no-host-path \
    > "$O/sortvar_$v.log" 2>&1 || { echo "variant $v failed"; tail -5 "$O/sortvar_$v.log"; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/sortvar_$v.log) $(grep -o '"phases_ms": {[^}]*' $O/sortvar_$v.log)"
done
SKV_LIB=skyvault-rs_amd/skv/variants/libskv_sortprof.so SKV_SORT_PROF_PRINT=1 timeout -k 10 300 python bench.py --config 5 \
  --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > "$O/sortprof.log" 2>&1 || { tail -5 "$O/sortprof.log"; exit 1; }
grep "sort prof" "$O/sortprof.log" | tail -4
