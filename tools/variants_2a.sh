#!/bin/bash
# Config-2A bench per library variant (SKV_LIB): ms per step and the k_fx_tile launch time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in base "$@"; do
  lib=skyvault-rs_amd/skv/libskv.so
  [ "$v" != base ] && lib=skyvault-rs_amd/skv/variants/libskv_$v.so
  SKV_LIB=$lib timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path \
    > gpurun_out/var_$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/var_$v.log) $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/var_$v.log)"
done
