#!/bin/bash
# Bench of one config under several env settings: KNOBS="A=1,B=2 C=3" (space-separated sets).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
C=${CONFIG:-3F}
i=0
for set in ${KNOBS:-none}; do
  i=$((i+1))
  envs=""; [ "$set" != none ] && envs=$(echo "$set" | tr ',' ' ')
  env $envs timeout -k 10 300 python bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/knob_${C}_$i.log 2>&1 || { echo "bench $set failed"; tail -5 gpurun_out/knob_${C}_$i.log; exit 1; }
  echo "$C [$set] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/knob_${C}_$i.log) $(grep -o '"phases_ms": {[^}]*}' gpurun_out/knob_${C}_$i.log)"
done
