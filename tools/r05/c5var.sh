#!/bin/bash
# Config 5 device line under env knobs: ENVS="tag:VAR=val,VAR=val tag2:..." (tag base = none).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05/c5var; mkdir -p $O
for spec in ${ENVS:-base:X=1}; do
  tag=${spec%%:*}; ev=${spec#*:}
  env ${ev//,/ } timeout -k 10 300 python bench.py --config 5 --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --no-host-path > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $O/$tag.log) $(grep -o '"phases_ms": {[^}]*' $O/$tag.log)"
done
