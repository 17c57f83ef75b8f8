#!/bin/bash
# One-pass span parse (skv_span.hip): general-path parity suites, then parse-phase A/B
# (SKV_SPAN=0 chunk walks vs the span parse) at config 3 (16 MiB runs) and 3F (256 MiB runs).
# Output: gpurun_out/r03/span_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03; mkdir -p $O
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_scan.py \
    tests/test_gpu_split.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/span_tests.log 2>&1 \
    || { tail -30 $O/span_tests.log; exit 1; }
  tail -2 $O/span_tests.log
fi
timeout -k 10 300 python -u tools/stage_probe.py SKV_SPAN=0 SKV_SPAN=1 > $O/span_probe16.log 2>&1 \
  || { tail -20 $O/span_probe16.log; exit 1; }
tail -2 $O/span_probe16.log
timeout -k 10 400 python -u tools/stage_probe.py --run-mib 256 SKV_SPAN=0 SKV_SPAN=1 > $O/span_probe256.log 2>&1 \
  || { tail -20 $O/span_probe256.log; exit 1; }
tail -2 $O/span_probe256.log
