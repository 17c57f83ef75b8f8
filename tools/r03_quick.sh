#!/bin/bash
# quick GPU check: TESTS (pytest args, -m gpu) then BENCHES (space-separated bench.py configs, 3 steps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03; mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TT:-600} python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $O/quick_tests.log 2>&1 \
    || { tail -30 $O/quick_tests.log; exit 1; }
  tail -2 $O/quick_tests.log
fi
for C in ${BENCHES:-}; do
  timeout -k 10 300 python -u bench.py --config $C --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-host-path > $O/quick_$C.json 2> $O/quick_$C.err \
    || { tail -20 $O/quick_$C.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/quick_$C.json'));print('$C', d['ms_per_step'], d['value'], d.get('phases_ms'))"
done
