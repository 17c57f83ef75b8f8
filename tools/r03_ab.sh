#!/bin/bash
# A/B of an env knob on one bench config: VAR=NAME, VALS="a b", CONFIG=3, REPS=2 (alternating)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03; mkdir -p $O
for r in $(seq 1 ${REPS:-2}); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python -u bench.py --config ${CONFIG:-3} --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-host-path \
      > $O/ab_${VAR}_$v.json 2> $O/ab_${VAR}_$v.err || { tail -20 $O/ab_${VAR}_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab_${VAR}_$v.json'));print('$VAR=$v', d['ms_per_step'], d['phases_ms'])"
  done
done
