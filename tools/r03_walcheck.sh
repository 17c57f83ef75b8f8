#!/bin/bash
# WAL stage check: parity / sort / jobs suites and the full-size config-5 test, then the config-5 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sort.py tests/test_jobs.py \
  tests/test_gpu_fullsize.py -k "not config3_full and not config2_full" -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/walcheck.log 2>&1 || { tail -40 $O/walcheck.log; exit 1; }
tail -2 $O/walcheck.log
BENCHES=5 bash tools/r03_quick.sh
