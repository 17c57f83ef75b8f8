#!/bin/bash
# Config-5 host timeline per SKV_HOST_THREADS value.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for t in ${THREADS:-8 16}; do
  SKV_HOST_THREADS=$t SKV_HOST_TRACE=1 timeout -k 10 200 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/ht5_$t.log 2>&1 || { echo "bench failed"; exit 1; }
  echo "threads $t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ht5_$t.log)"
  grep "skv host" gpurun_out/ht5_$t.log | tail -17 | tr '\n' ' ' | sed 's/\[skv host\]//g'; echo
done
