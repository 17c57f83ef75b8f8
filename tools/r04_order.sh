#!/bin/bash
# The order check fused into k_emit (SKV_EMIT_ORDER=1, default) against k_order_check (=0): the
# general-path parity files, then configs 3 and 3F timed both ways. Output: gpurun_out/r04/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="$PWD/gpurun_out/r04"
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_scan.py tests/test_gpu_hostpipe.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > "$O/order_tests.log" 2>&1
rc=$?
tail -2 "$O/order_tests.log"
[ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)" "$O/order_tests.log" | head -20; exit $rc; }
for c in 3 3F; do
  for v in 0 1; do
    SKV_EMIT_ORDER=$v timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline \
      --no-host-path > "$O/order_${c}_$v.log" 2>&1 || { echo "bench $c $v failed"; tail -5 "$O/order_${c}_$v.log"; exit 1; }
    echo "$c emit_order=$v $(grep -o '"ms_per_step": [0-9.]*' $O/order_${c}_$v.log) $(grep -o '"phases_ms": {[^}]*' $O/order_${c}_$v.log)"
  done
done
