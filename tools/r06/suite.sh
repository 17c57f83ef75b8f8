#!/bin/bash
# the whole GPU suite (the driver's round-end command), log under gpurun_out/r06/suite/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O="$PWD/gpurun_out/r06/suite"; mkdir -p "$O"
timeout -k 10 1100 python3 -u -m pytest tests/ -x -q -m gpu --timeout 600 --timeout-method thread ${PYARGS:-} > "$O/suite.log" 2>&1
rc=$?; tail -8 "$O/suite.log"; exit $rc
