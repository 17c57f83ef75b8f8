#!/bin/bash
# Config 5 step time by host pool size (SKV_HOST_THREADS) with the host-side trace of one call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="$PWD/gpurun_out/r04"
mkdir -p "$O"
for t in ${THREADS:-4 8 16}; do
  env ${EXTRA_ENV:-SKV_NONE=1} SKV_HOST_THREADS=$t timeout -k 10 300 python bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline --no-host-path \
    > "$O/hthreads_$t.log" 2>&1 || { echo "threads $t failed"; tail -5 "$O/hthreads_$t.log"; exit 1; }
  echo "threads $t $(grep -o '"ms_per_step": [0-9.]*' $O/hthreads_$t.log) $(grep -o '"host_ms": {[^}]*' $O/hthreads_$t.log)"
  env ${EXTRA_ENV:-SKV_NONE=1} SKV_HOST_TRACE=1 SKV_HOST_THREADS=$t timeout -k 10 300 python bench.py --config 5 --steps 1 --warmup 1 --no-cpu-baseline \
    --no-host-path > "$O/hthreads_trace_$t.log" 2>&1 || exit 1
  grep "skv host" "$O/hthreads_trace_$t.log" | tail -12 | head -7 | tr '\n' ' '; echo
done
