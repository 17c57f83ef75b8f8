#!/bin/bash
# General merge-tile variants on configs 3 and 3F (tools/build_variants_r04.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="$PWD/gpurun_out/r04"
mkdir -p "$O"
for c in ${CONFIGS_T:-3 3F}; do
  for v in ${VARIANTS:-base t512}; do
    lib=skyvault-rs_amd/skv/libskv.so
    [ "$v" != base ] && lib=skyvault-rs_amd/skv/variants/libskv_$v.so
    SKV_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-host-path \
      > "$O/tilevar_${c}_$v.log" 2>&1 || { echo "variant $v $c failed"; tail -5 "$O/tilevar_${c}_$v.log"; exit 1; }
    echo "$c $v $(grep -o '"ms_per_step": [0-9.]*' $O/tilevar_${c}_$v.log) $(grep -o '"phases_ms": {[^}]*' $O/tilevar_${c}_$v.log)"
  done
done
