#!/bin/bash
# Non-slow GPU suite, then the bench of the configs given (default 3 3F): ms per step and phases.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/chk_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/chk_tests.log; exit 1; }
tail -1 gpurun_out/chk_tests.log
for C in ${CONFIGS:-3 3F}; do
  timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-host-path \
    > gpurun_out/chk_$C.log 2>&1 || { echo "bench $C failed"; exit 1; }
  echo "$C $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/chk_$C.log) $(grep -o '"phases_ms": {[^}]*}' gpurun_out/chk_$C.log)"
done
