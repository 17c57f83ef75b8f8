#!/bin/bash
# Round-5 check on one MI355X: the -m gpu suite (per-test timeout, thread method), then the
# default bench line. Output: gpurun_out/r05/. TESTS=<pytest args> narrows the suite; MARK
# overrides the marker expression; BENCH=0 skips the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O="$PWD/gpurun_out/r05"
mkdir -p "$O"
timeout -k 10 ${TLIM:-1000} python -u -m pytest ${TESTS:-tests} -m "${MARK:-gpu}" -v --timeout 300 --timeout-method thread \
  > "$O/tests${TAG:-}.log" 2>&1
rc=$?
tail -5 "$O/tests${TAG:-}.log"
[ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)|(FAILED|ERROR) " "$O/tests${TAG:-}.log" | head -30; exit $rc; }
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python bench.py > "$O/bench${TAG:-}.log" 2>&1 || { tail -20 "$O/bench${TAG:-}.log"; exit 1; }
  tail -1 "$O/bench${TAG:-}.log" | cut -c1-700
fi
exit 0
