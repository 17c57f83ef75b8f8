#!/bin/bash
# Config-5 bench per library variant (VARS="base k4i2 ..."), kernel time of k_sort_bucket from the phases.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARS:-base}; do
  lib=skyvault-rs_amd/skv/libskv.so
  [ "$v" != base ] && lib=skyvault-rs_amd/skv/variants/libskv_$v.so
  SKV_LIB=$lib timeout -k 10 200 python bench.py --config ${CONFIG:-5} --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/v5_$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/v5_$v.log) $(grep -o '"merge": [0-9.]*' gpurun_out/v5_$v.log)"
done
