#!/bin/bash
# Round-4 check on one MI355X: the whole -m gpu suite (per-test timeout, thread method), then the
# default bench line. Output: gpurun_out/r04/. TESTS=<pytest args> narrows the suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="$PWD/gpurun_out/r04"
mkdir -p "$O"
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -q --timeout 300 --timeout-method thread \
  > "$O/tests${TAG:-}.log" 2>&1
rc=$?
tail -5 "$O/tests${TAG:-}.log"
[ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)" "$O/tests${TAG:-}.log" | head -30; exit $rc; }
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python bench.py > "$O/bench${TAG:-}.log" 2>&1 || { tail -20 "$O/bench${TAG:-}.log"; exit 1; }
  tail -1 "$O/bench${TAG:-}.log" | cut -c1-600
fi
exit 0
