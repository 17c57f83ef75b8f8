#!/bin/bash
# Round-2 experiment session: sort/WAL parity tests, config-5 bench, config-2A cache-policy variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/exp_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/exp_tests.log; exit 1; }
tail -1 gpurun_out/exp_tests.log
timeout -k 10 200 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/exp_5.log 2>&1 || { echo "bench 5 failed"; exit 1; }
echo "5 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/exp_5.log) $(grep -o '"phases_ms": {[^}]*}' gpurun_out/exp_5.log)"
for spec in ${VARIANTS:-}; do
  v=${spec%%:*}; lds=${spec#*:}
  lib=skyvault-rs_amd/skv/libskv.so
  [ "$v" != base ] && lib=skyvault-rs_amd/skv/variants/libskv_$v.so
  SKV_FX_LDS=$lds SKV_LIB=$lib timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path \
    > gpurun_out/exp_var_${v}_$lds.log 2>&1 || { echo "variant $spec failed"; exit 1; }
  echo "$spec $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/exp_var_${v}_$lds.log) $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/exp_var_${v}_$lds.log)"
done
